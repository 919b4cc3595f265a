"""PPE multi-label activity classifier: the reference's second DDP application, made runnable.

Reference: ``ppe_main_ddp.py``.  As shipped it cannot run: its model (``model.ResNet101``),
dataset (``datasets.ppe_io.PPE``), preprocessing and ``evaluate_map.compute_map`` modules are missing, and it
needs cv2 / lxml / ``scipy.misc.imread`` (all absent here).  This module provides every piece, so the same
workflow runs on MI355X:

* ``PPEDataset``: images (``.png/.jpg/.npy``) with Pascal-VOC XML labels (``xml.etree``, no lxml) giving person
  boxes and 3 binary activity attributes, resized to 120 x 160 (the reference's ``img_shape``); or
  ``synthetic_ppe()`` for offline runs.  Items are ``(image[3,120,160], boxes[n,4], labels[n,3], path)``;
  ``detection_collate`` makes ``(images, bboxes[N,5] = (batch_idx, x1, y1, x2, y2), labels[N,3], paths)``.
* ``ResNet101ROI``: the ResNet-101 trunk (``models/resnet50.py``) + ROI-align over the stride-16 features
  (bilinear ``grid_sample``, 4x4 bins) + a 3-way multi-label head.  This is the ``model(data, bboxes)`` contract
  of ``ppe_main_ddp.py:146``.  On GPU every conv / BN / pool / fc runs on the ops layer's HIP kernels
  (``OpsModel.begin/stem/blocks/head``); ``engine="torch"`` keeps the stock torch modules.
* ``train`` (``:128-182``): SGD(1e-3, momentum 0.9) via ``FlatSGD``, BCE-with-logits, progress print every 100
  iterations, ``model-ep{E}.pth`` every 5 epochs (rank 0), validation loss per epoch, loss-curve PNG.
* ``eval_model`` / ``compute_map`` / ``plot_graph`` (``:186-231``): per-class AP (area under the interpolated
  precision-recall curve), mAP, PR-curve PNG.
* ``k_fold_cv`` (``:234-307``): k-fold cross-validation with fresh models per fold and a per-fold summary.
* ``pre_generate_labels`` (``:310-396``): inference that writes box-annotated images and a JSON of boxes/scores.

Deliberate fixes: ``-freeze`` really freezes (``requires_grad``, applied before the DDP
wrap); k-fold calls ``train`` with the right arguments; validation runs in eval mode and averages every val batch
(the reference kept only the last).  ``pre_generate_labels`` keeps the reference's raw-logit threshold and 0/1
"scores" (as floats 0.0 / 1.0, like its ``pred.astype(np.float)``); ``with_probs=True`` adds the sigmoid
probabilities as "probs" (an extension).
"""
from __future__ import annotations

import json
import os
import time
import xml.etree.ElementTree as ET
from statistics import mean
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..models.resnet50 import ResNet, Bottleneck

IMG_SHAPE = (120, 160)  # (H, W), reference ppe_main_ddp.py:74
TARGETS = {"rc_nc_ma": ["rc", "nc", "ma"], "ca_ea_ma": ["ca", "ea", "ma"]}
PIX_MEAN = (0.485, 0.456, 0.406)
PIX_STD = (0.229, 0.224, 0.225)


# ---------------------------------------------------------------------------------------------------------------
# data
class PPEDataset(torch.utils.data.Dataset):
    def __init__(self, img_root: str, label_root: str, target: str = "rc_nc_ma", img_shape=IMG_SHAPE):
        self.img_root, self.label_root, self.img_shape = img_root, label_root, img_shape
        self.attrs = TARGETS[target]
        exts = (".png", ".jpg", ".jpeg", ".npy")
        self.files = sorted(f for f in os.listdir(img_root) if f.lower().endswith(exts))

    def __len__(self) -> int:
        return len(self.files)

    def _load_image(self, path: str) -> np.ndarray:
        if path.endswith(".npy"):
            return np.load(path, allow_pickle=False)
        from PIL import Image
        return np.asarray(Image.open(path).convert("RGB"))

    def __getitem__(self, i: int):
        path = os.path.join(self.img_root, self.files[i])
        img = self._load_image(path)
        h0, w0 = img.shape[:2]
        x = torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1).float()[None]
        x = F.interpolate(x, size=self.img_shape, mode="bilinear", align_corners=False)[0]
        boxes, labels = [], []
        xml = os.path.join(self.label_root, os.path.splitext(self.files[i])[0] + ".xml")
        if os.path.exists(xml):
            root = ET.parse(xml).getroot()
            sy, sx = self.img_shape[0] / h0, self.img_shape[1] / w0
            for obj in root.iter("object"):
                bb = obj.find("bndbox")
                if bb is None:
                    continue
                x1, y1, x2, y2 = (float(bb.find(k).text) for k in ("xmin", "ymin", "xmax", "ymax"))
                boxes.append([x1 * sx, y1 * sy, x2 * sx, y2 * sy])
                labels.append([1.0 if (obj.find(a) is not None and obj.find(a).text.strip() in ("1", "true"))
                               else 0.0 for a in self.attrs])
        if not boxes:  # the reference pads images without persons with a dummy 10x10 box
            boxes, labels = [[0.0, 0.0, 10.0, 10.0]], [[0.0] * len(self.attrs)]
        return x, torch.tensor(boxes), torch.tensor(labels), path

    @staticmethod
    def detection_collate(batch):
        imgs, bbs, lbs, paths = [], [], [], []
        for bi, (x, b, l, p) in enumerate(batch):
            imgs.append(x)
            bbs.append(torch.cat([torch.full((len(b), 1), float(bi)), b], 1))
            lbs.append(l)
            paths.append(p)
        return torch.stack(imgs), torch.cat(bbs), torch.cat(lbs), paths


class SyntheticPPE(torch.utils.data.Dataset):
    """Offline stand-in: random images with 1-4 random person boxes whose attributes depend on the box contents
    (so the task is learnable), 120 x 160."""

    def __init__(self, n: int = 256, seed: int = 0, n_attr: int = 3):
        g = torch.Generator().manual_seed(seed)
        self.items = []
        H, W = IMG_SHAPE
        for i in range(n):
            x = torch.rand(3, H, W, generator=g) * 255
            k = int(torch.randint(1, 5, (1,), generator=g))
            boxes, labels = [], []
            for _ in range(k):
                w = float(torch.randint(16, 64, (1,), generator=g))
                h = float(torch.randint(24, 80, (1,), generator=g))
                x1 = float(torch.randint(0, int(W - w), (1,), generator=g))
                y1 = float(torch.randint(0, int(H - h), (1,), generator=g))
                lab = (torch.rand(n_attr, generator=g) > 0.5).float()
                for a in range(n_attr):  # paint the evidence into the box: channel a bright iff attribute a
                    x[a, int(y1):int(y1 + h), int(x1):int(x1 + w)] = 230.0 if lab[a] > 0 else 20.0
                boxes.append([x1, y1, x1 + w, y1 + h])
                labels.append(lab)
            self.items.append((x, torch.tensor(boxes), torch.stack(labels), f"synthetic_{i:05d}"))

    def __len__(self) -> int:
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]

    detection_collate = staticmethod(PPEDataset.detection_collate)


def preprocess_img(x: torch.Tensor) -> torch.Tensor:
    """uint8-range RGB -> ImageNet-normalised (the missing reference datasets.transform.preprocess_img)."""
    mean_ = torch.tensor(PIX_MEAN, device=x.device).view(1, 3, 1, 1)
    std_ = torch.tensor(PIX_STD, device=x.device).view(1, 3, 1, 1)
    return (x / 255.0 - mean_) / std_


# ---------------------------------------------------------------------------------------------------------------
# model
class ResNet101ROI(nn.Module):
    """ResNet-101 trunk to stride 16 (layer1-3) + ROI-align of every box + layer4 + multi-label head."""

    def __init__(self, num_classes: int = 3, bins: int = 4, layers: Sequence[int] = (3, 4, 23, 3),
                 engine: str = "auto"):
        super().__init__()
        if engine not in ("auto", "ops", "torch"):
            raise ValueError(f"engine {engine!r}: auto | ops | torch")
        self.engine = engine  # auto: the ops layer's HIP kernels on GPU, torch modules on CPU
        r = ResNet(list(layers), num_classes=1000, zero_init_residual=False)  # (1,1,1,1) for tests
        self.stem = nn.Sequential(r.conv1, r.bn1, r.relu, r.maxpool)
        self.layer1, self.layer2, self.layer3, self.layer4 = r.layer1, r.layer2, r.layer3, r.layer4
        self.fc = nn.Linear(512 * Bottleneck.expansion, num_classes)
        self.bins = bins

    def roi_align(self, feat: torch.Tensor, boxes: torch.Tensor, stride: float) -> torch.Tensor:
        """feat [B,C,h,w], boxes [N,5] (batch_idx, x1, y1, x2, y2 in input pixels) -> [N,C,bins,bins]."""
        n, k = boxes.shape[0], self.bins
        bi = boxes[:, 0].long()
        h, w = feat.shape[-2:]
        t = (torch.arange(k, device=feat.device, dtype=feat.dtype) + 0.5) / k
        xs = boxes[:, 1:2] + (boxes[:, 3:4] - boxes[:, 1:2]) * t          # [N,k] pixel x
        ys = boxes[:, 2:3] + (boxes[:, 4:5] - boxes[:, 2:3]) * t
        gx = (xs / stride) / w * 2 - 1                                    # normalised, align_corners=False
        gy = (ys / stride) / h * 2 - 1
        grid = torch.stack([gx[:, None, :].expand(n, k, k), gy[:, :, None].expand(n, k, k)], -1)
        return F.grid_sample(feat[bi], grid, mode="bilinear", padding_mode="border", align_corners=False)

    def forward(self, x: torch.Tensor, boxes: torch.Tensor) -> torch.Tensor:
        if x.is_cuda and self.engine != "torch":
            return self._forward_ops(x, boxes)
        if self.engine == "ops":
            raise RuntimeError("ResNet101ROI(engine='ops') needs a GPU input")
        f = self.layer3(self.layer2(self.layer1(self.stem(x))))          # stride 16
        r = self.layer4(self.roi_align(f, boxes.to(f.dtype), 16.0))     # [N,2048,2,2]
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(r, 1), 1))

    def _forward_ops(self, x: torch.Tensor, boxes: torch.Tensor) -> torch.Tensor:
        """The same network on the ops layer's HIP kernels (implicit-GEMM MFMA convs with the BN statistics in
        the epilogue, fused BN + ReLU + residual, pools, fc) over NHWC bf16 activations.  Only the ROI gather
        (bilinear ``grid_sample`` of a few boxes per image) stays in torch.  Training-mode BN trains; eval mode
        is the inference path (running statistics, under no_grad)."""
        ops = self.__dict__.get("_ops")
        if ops is None:  # kept out of the module tree: OpsModel wraps this module (no state_dict cycle)
            from ..ops import OpsModel
            ops = self.__dict__["_ops"] = OpsModel(self)
        h = ops.begin(x)
        h = ops.stem(h, self.stem[0], self.stem[1])
        h = ops.blocks(h, [*self.layer1, *self.layer2, *self.layer3])             # stride 16, NHWC bf16
        r = self.roi_align(h.permute(0, 3, 1, 2).float(), boxes.float(), 16.0)  # [N,1024,bins,bins] fp32
        h = ops.blocks(r.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous(), self.layer4)
        return ops.head(h, self.fc)


def freeze_backbone(model: nn.Module) -> None:
    """-freeze: only layer4.2 and fc train (reference intent, ppe_main_ddp.py:117-122; typo fixed)."""
    for name, p in model.named_parameters():
        p.requires_grad = ("layer4.2" in name) or name.startswith("fc")


def build_model(load_model: Optional[str] = None, num_classes: int = 3,
                layers: Sequence[int] = (3, 4, 23, 3), engine: str = "auto") -> nn.Module:
    m = ResNet101ROI(num_classes, layers=layers, engine=engine)
    if load_model and os.path.exists(load_model):
        sd = torch.load(load_model, map_location="cpu", weights_only=True)
        sd = {k: v for k, v in sd.items() if not (k.startswith("fc.") and v.shape[0] != num_classes)}
        m.load_state_dict(sd, strict=False)
    return m


# ---------------------------------------------------------------------------------------------------------------
# metrics
def compute_map(pred: np.ndarray, gt: np.ndarray, num_classes: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Per-class average precision (area under the monotone precision envelope), and the curves sampled at 101
    recall points: (AP[C], prec[C,101], rec[C,101])."""
    ap = np.zeros(num_classes)
    rgrid = np.linspace(0, 1, 101)
    prec_all = np.zeros((num_classes, 101))
    for c in range(num_classes):
        order = np.argsort(-pred[:, c], kind="stable")
        tp = gt[order, c] > 0.5
        npos = max(int(tp.sum()), 1)
        ctp, cfp = np.cumsum(tp), np.cumsum(~tp)
        rec = ctp / npos
        prec = ctp / np.maximum(ctp + cfp, 1)
        mrec = np.concatenate([[0.0], rec, [1.0]])
        mpre = np.concatenate([[1.0], prec, [0.0]])
        for i in range(len(mpre) - 2, -1, -1):
            mpre[i] = max(mpre[i], mpre[i + 1])
        idx = np.where(mrec[1:] != mrec[:-1])[0]
        ap[c] = float(np.sum((mrec[idx + 1] - mrec[idx]) * mpre[idx + 1]))
        prec_all[c] = np.interp(rgrid, mrec, mpre, right=0.0)
    return ap, prec_all, np.tile(rgrid, (num_classes, 1))


def _savefig(path: str, draw) -> None:
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    plt.figure()
    draw(plt)
    plt.savefig(path)
    plt.close()


def plot_graph(AP, prec_all, rec_all, save_dir: str, target_list: Sequence[str]) -> str:
    path = os.path.join(save_dir, "precision-recall-curve.png")

    def draw(plt):
        for i in range(prec_all.shape[0]):
            plt.plot(rec_all[i], prec_all[i], label="{} AP = {:.5f}".format(target_list[i], AP[i]))
        plt.xlabel("Recall")
        plt.ylabel("Precision")
        plt.title("model performance: mAP = {:.3f}".format(float(np.mean(AP))))
        plt.legend()
    _savefig(path, draw)
    return path


# ---------------------------------------------------------------------------------------------------------------
# training / evaluation
def _batches(loader, device):
    for data, bboxes, labels, paths in loader:
        yield preprocess_img(data.float().to(device)), bboxes.to(device), labels.to(device), paths


def train(data_loader, data_loader_eval, model, save_dir: str, num_epoch: int, rank: int = 0, lr: float = 1e-3,
          device=None, max_iters: Optional[int] = None):
    """Reference ppe_main_ddp.py:128-182.  `model` is a FlatBucketDDP (or a plain module)."""
    from ..parallel.flat_ddp import FlatBucketDDP, FlatSGD
    device = device or next(model.parameters()).device
    os.makedirs(save_dir, exist_ok=True)
    print("=========================================")
    print("start training")
    opt = FlatSGD(model, lr=lr, momentum=0.9) if isinstance(model, FlatBucketDDP) else \
        torch.optim.SGD([p for p in model.parameters() if p.requires_grad], lr=lr, momentum=0.9)
    train_losses, val_losses = [], []
    start = time.time()
    inner = getattr(model, "module", model)
    for epoch in range(num_epoch + 1):
        model.train()
        it, loss = 0, torch.zeros(())
        for data, bboxes, labels, _ in _batches(data_loader, device):
            it += 1
            opt.zero_grad()
            loss = F.binary_cross_entropy_with_logits(model(data, bboxes), labels)
            loss.backward()
            opt.step()
            if it % 100 == 0:
                print("epoch {} iterate {} train loss {}".format(epoch, it, loss.item()))
            if max_iters and it >= max_iters:
                break
        train_losses.append(float(loss.item()))
        if hasattr(model, "check_comm"):  # FlatBucketDDP over xGMI: a peer timeout must raise, not diverge
            model.check_comm()
        if (epoch % 5 == 0 or epoch == 100) and rank == 0:
            torch.save(inner.state_dict(), os.path.join(save_dir, "model-ep{}.pth".format(epoch)))
            print("model is saved in", save_dir)
        model.eval()
        vl = []
        with torch.no_grad():
            for data, bboxes, labels, _ in _batches(data_loader_eval, device):
                vl.append(float(F.binary_cross_entropy_with_logits(model(data, bboxes), labels)))
        val_losses.append(mean(vl) if vl else float("nan"))
        print("=========================================")
        print("epoch {} train loss {:.5f} val loss {:.5f}".format(epoch, train_losses[epoch], val_losses[epoch]))
        print("=========================================")
    print(f"training time: {time.time() - start:.3f} seconds")
    if rank == 0:
        def draw(plt):
            plt.plot(train_losses, label="Training Loss")
            plt.plot(val_losses, label="Validation Loss")
            plt.legend()
            plt.title("Loss loss curve")
        _savefig(os.path.join(save_dir, "loss_graph.png"), draw)
    return mean(train_losses), mean(val_losses)


def eval_model(model, data_loader_eval, save_dir: str, target_list: Sequence[str], device=None):
    """Reference ppe_main_ddp.py:186-221: per-class AP, mAP, PR curves."""
    device = device or next(model.parameters()).device
    print("=========================================")
    print("start eval")
    preds, gts = [], []
    model.eval()
    with torch.no_grad():
        for data, bboxes, labels, _ in _batches(data_loader_eval, device):
            preds.append(torch.sigmoid(model(data, bboxes)).float().cpu().numpy())
            gts.append(labels.cpu().numpy())
    pred, gt = np.concatenate(preds), np.concatenate(gts)
    AP, prec_all, rec_all = compute_map(pred, gt, len(target_list))
    mAP = float(np.mean(AP))
    for i in range(len(target_list)):
        print(target_list[i], "AP = {}".format(AP[i]))
    print("mAP = {}".format(mAP))
    os.makedirs(save_dir, exist_ok=True)
    plot_graph(AP, prec_all, rec_all, save_dir, target_list)
    return (mAP, *[float(a) for a in AP])


def k_fold_cv(dataset, k: int, load_model: Optional[str], save_dir: str, num_epoch: int, target_list: List[str],
              freeze_opt: bool, device, batch_size: int = 2, max_iters: Optional[int] = None,
              layers: Sequence[int] = (3, 4, 23, 3)):
    """Reference ppe_main_ddp.py:234-307 (single process; the reference's call bug fixed)."""
    n = len(dataset)
    fold = n // k
    idx = list(range(n))
    res = {"train": [], "val": [], "mAP": [], "AP": []}
    for f in range(k):
        print("==================fold {}==================".format(f))
        model = build_model(load_model, len(target_list), layers)
        if freeze_opt:
            freeze_backbone(model)
        model.to(device)
        tr = idx[:f * fold] + idx[(f + 1) * fold:]
        va = idx[f * fold:(f + 1) * fold]
        mk = lambda ids: torch.utils.data.DataLoader(  # noqa: E731
            dataset, batch_size=batch_size, sampler=torch.utils.data.SubsetRandomSampler(ids),
            collate_fn=dataset.detection_collate, drop_last=True)
        path = os.path.join(save_dir, "fold{}".format(f))
        tl, vl = train(mk(tr), mk(va), model, path, num_epoch, 0, device=device, max_iters=max_iters)
        print("average training loss for fold{}: {:.5f}".format(f, tl))
        print("average validation loss for fold{}: {:.5f}".format(f, vl))
        mAP, *aps = eval_model(model, mk(va), path, target_list, device)
        res["train"].append(round(tl, 5))
        res["val"].append(round(vl, 5))
        res["mAP"].append(round(mAP, 5))
        res["AP"].append([round(a, 5) for a in aps])
    print("train loss for each fold: {}".format(res["train"]))
    print("validation loss for each fold: {}".format(res["val"]))
    print("mAP for each fold: {}".format(res["mAP"]))
    for i, t in enumerate(target_list):
        print("{} AP for each fold: {}".format(t, [a[i] for a in res["AP"]]))
    return res


def pre_generate_labels(model, dataset, model_name: Optional[str], out_dir: str = "outputs",
                        json_path: str = "PPE_preds_160.json", threshold: float = 0.5, device=None,
                        threshold_probs: bool = False, with_probs: bool = False):
    """Reference ppe_main_ddp.py:310-396: predict every box, draw the boxes with their active attributes onto
    the image, write the images and a JSON of boxes / scores.

    As the reference (its sigmoid is commented out), an attribute is on when its RAW LOGIT exceeds `threshold`,
    and the JSON "scores" are those decisions as 0.0 / 1.0; ``with_probs`` adds the sigmoid probabilities.
    ``threshold_probs=True`` thresholds the probabilities instead (logit > logit(threshold))."""
    from PIL import Image, ImageDraw
    device = device or next(model.parameters()).device
    if model_name:
        assert os.path.isfile(model_name), f"no checkpoint at {model_name}"
        model.load_state_dict(torch.load(model_name, map_location="cpu", weights_only=True))
    os.makedirs(out_dir, exist_ok=True)
    attrs = ["rc", "nc", "ma"]
    out = {}
    model.eval()
    with torch.no_grad():
        for i in range(len(dataset)):
            img, boxes, _, path = dataset[i]
            bb = torch.cat([torch.zeros(len(boxes), 1), boxes], 1)
            logits = model(preprocess_img(img[None].to(device)), bb.to(device)).float().cpu()
            probs = torch.sigmoid(logits).numpy()
            p = ((probs if threshold_probs else logits.numpy()) > threshold).astype(np.int64)
            name = os.path.splitext(os.path.basename(str(path)))[0]
            # the reference writes pred.astype(np.float): 0.0 / 1.0 (ppe_main_ddp.py:368); probabilities only
            # on request (an extension of the reference's format)
            out[name] = {"bboxes": boxes.tolist(), "scores": p.astype(np.float64).tolist()}
            if with_probs:
                out[name]["probs"] = probs.tolist()
            canvas = Image.fromarray(img.permute(1, 2, 0).clamp(0, 255).byte().numpy())
            draw = ImageDraw.Draw(canvas)
            for (x1, y1, x2, y2), s in zip(boxes.tolist(), p):
                if x2 - x1 == 10 and y2 - y1 == 10:  # padding box of person-free frames
                    continue
                draw.rectangle([x1, y1, x2, y2], outline=(0, 255, 0), width=2)
                draw.text((x1, max(y1 - 10, 0)), "h" + "".join(f"_{a}" for a, v in zip(attrs, s) if v),
                          fill=(255, 0, 0))
            canvas.save(os.path.join(out_dir, f"{name}.jpg"))
    with open(json_path, "w") as f:
        json.dump(out, f)
    return out
