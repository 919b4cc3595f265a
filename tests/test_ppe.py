"""PPE application (reference ppe_main_ddp.py): data, ROI model, metrics, train/eval/k-fold,
label generation and the DDP entry point (gloo, 2 ranks)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from distributeddataparallel_cifar10_amd.apps import ppe

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = (1, 1, 1, 1)


def _write_sample(d, name, boxes, attrs, shape=(240, 320)):
    os.makedirs(os.path.join(d, "img"), exist_ok=True)
    os.makedirs(os.path.join(d, "lab"), exist_ok=True)
    np.save(os.path.join(d, "img", name + ".npy"), np.full(shape + (3,), 100, np.uint8))
    objs = "".join(
        "<object><name>person</name><bndbox><xmin>{}</xmin><ymin>{}</ymin><xmax>{}</xmax><ymax>{}</ymax></bndbox>"
        "<rc>{}</rc><nc>{}</nc><ma>{}</ma></object>".format(*b, *a) for b, a in zip(boxes, attrs))
    with open(os.path.join(d, "lab", name + ".xml"), "w") as f:
        f.write(f"<annotation><filename>{name}</filename>{objs}</annotation>")


def test_dataset_xml_and_resize(tmp_path):
    _write_sample(str(tmp_path), "a", [(20, 40, 100, 200), (0, 0, 320, 240)], [(1, 0, 1), (0, 1, 0)])
    _write_sample(str(tmp_path), "b", [], [])
    ds = ppe.PPEDataset(str(tmp_path / "img"), str(tmp_path / "lab"))
    assert len(ds) == 2
    x, b, l, p = ds[0]
    assert x.shape == (3, 120, 160) and torch.allclose(x, torch.full_like(x, 100.0))
    assert torch.allclose(b, torch.tensor([[10.0, 20.0, 50.0, 100.0], [0.0, 0.0, 160.0, 120.0]]))
    assert l.tolist() == [[1, 0, 1], [0, 1, 0]]
    _, b2, l2, _ = ds[1]  # no persons -> one 10x10 padding box, all-zero labels
    assert b2.tolist() == [[0, 0, 10, 10]] and l2.tolist() == [[0, 0, 0]]
    imgs, bb, ll, paths = ppe.PPEDataset.detection_collate([ds[0], ds[1]])
    assert imgs.shape == (2, 3, 120, 160) and bb.shape == (3, 5) and ll.shape == (3, 3)
    assert bb[:, 0].tolist() == [0, 0, 1]


def test_roi_align_matches_bilinear():
    m = ppe.ResNet101ROI(3, layers=TINY)
    feat = torch.randn(2, 5, 8, 10, dtype=torch.float64)
    # a box whose 4x4 bin centres land exactly on feature-pixel centres (stride 16): x 16..80, y 32..96
    boxes = torch.tensor([[1, 16.0, 32.0, 80.0, 96.0]], dtype=torch.float64)
    r = m.roi_align(feat, boxes, 16.0)
    # bin centre i -> pixel x = 16 + 64*(i+.5)/4 = 24 + 16 i -> feature coord (x/16 - 0.5) = 1 + i
    ref = feat[1, :, 1 + 1:1 + 1 + 4, 1:1 + 4]
    assert r.shape == (1, 5, 4, 4)
    torch.testing.assert_close(r[0], ref)


def test_model_forward_backward_and_freeze():
    m = ppe.ResNet101ROI(3, layers=TINY)
    x = torch.randn(2, 3, 120, 160)
    boxes = torch.tensor([[0, 0, 0, 50, 80], [1, 10, 10, 150, 110], [1, 0, 0, 10, 10]], dtype=torch.float)
    out = m(x, boxes)
    assert out.shape == (3, 3)
    torch.nn.functional.binary_cross_entropy_with_logits(out, torch.ones(3, 3)).backward()
    assert m.layer1[0].conv1.weight.grad is not None
    full = ppe.ResNet101ROI(3)
    assert sum(p.numel() for p in full.parameters()) > 40_000_000  # ResNet-101 trunk
    ppe.freeze_backbone(full)
    trainable = {n for n, p in full.named_parameters() if p.requires_grad}
    assert trainable and all(n.startswith("layer4.2") or n.startswith("fc") for n in trainable)
    assert "fc.weight" in trainable and "layer4.2.conv3.weight" in trainable


def test_compute_map():
    gt = np.array([[1, 0], [1, 1], [0, 0], [0, 1]], float)
    perfect = np.array([[0.9, 0.1], [0.8, 0.9], [0.1, 0.2], [0.2, 0.8]])
    ap, prec, rec = ppe.compute_map(perfect, gt, 2)
    assert np.allclose(ap, 1.0) and prec.shape == (2, 101) and rec.shape == (2, 101)
    # ranking + - + - : envelope precision 1 at recall .5, 2/3 at recall 1 -> AP = .5*1 + .5*2/3
    pred = np.array([[0.9], [0.1], [0.7], [0.8]])
    ap, _, _ = ppe.compute_map(pred, np.array([[1], [1], [0], [0]], float), 1)
    assert ap[0] == pytest.approx(0.5 + 0.5 * 0.5)
    sk = pytest.importorskip("sklearn.metrics")
    rng = np.random.default_rng(0)
    g = (rng.random((200, 3)) > 0.6).astype(float)
    p = rng.random((200, 3)) + 0.5 * g
    ap, _, _ = ppe.compute_map(p, g, 3)
    for c in range(3):  # the interpolated envelope never lies below the step AP
        assert ap[c] >= sk.average_precision_score(g[:, c], p[:, c]) - 1e-12


def test_train_eval_kfold_pregenerate(tmp_path):
    ds = ppe.SyntheticPPE(8, seed=0)
    dl = torch.utils.data.DataLoader(ds, batch_size=2, collate_fn=ds.detection_collate, drop_last=True)
    model = ppe.build_model(None, 3, TINY)
    tl, vl = ppe.train(dl, dl, model, str(tmp_path / "run"), 0, 0, device=torch.device("cpu"), max_iters=2)
    assert np.isfinite(tl) and np.isfinite(vl)
    assert (tmp_path / "run" / "model-ep0.pth").exists() and (tmp_path / "run" / "loss_graph.png").exists()
    sd = torch.load(tmp_path / "run" / "model-ep0.pth", weights_only=True)
    assert set(sd) == set(model.state_dict())
    res = ppe.eval_model(model, dl, str(tmp_path / "run"), ["rc", "nc", "ma"])
    assert len(res) == 4 and (tmp_path / "run" / "precision-recall-curve.png").exists()
    cv = ppe.k_fold_cv(ds, 2, None, str(tmp_path / "cv"), 0, ["rc", "nc", "ma"], True, torch.device("cpu"),
                       batch_size=2, max_iters=1, layers=TINY)
    assert len(cv["mAP"]) == 2 and len(cv["AP"][0]) == 3
    out = ppe.pre_generate_labels(model, ppe.SyntheticPPE(2, seed=3), str(tmp_path / "run" / "model-ep0.pth"),
                                  out_dir=str(tmp_path / "out"), json_path=str(tmp_path / "p.json"))
    assert len(out) == 2 and len(os.listdir(tmp_path / "out")) == 2
    j = json.load(open(tmp_path / "p.json"))
    k = next(iter(j))
    assert len(j[k]["bboxes"]) == len(j[k]["scores"]) and len(j[k]["scores"][0]) == 3
    # reference: pred.astype(np.float) of the raw-logit decisions -> 0.0 / 1.0 floats, no "probs" key
    assert {v for row in j[k]["scores"] for v in row} <= {0.0, 1.0}
    assert all(isinstance(v, float) for row in j[k]["scores"] for v in row) and "probs" not in j[k]
    out = ppe.pre_generate_labels(model, ppe.SyntheticPPE(2, seed=3), str(tmp_path / "run" / "model-ep0.pth"),
                                  out_dir=str(tmp_path / "out2"), json_path=str(tmp_path / "p2.json"), with_probs=True)
    j = json.load(open(tmp_path / "p2.json"))
    assert len(j[k]["probs"]) == len(j[k]["scores"])


def test_synthetic_is_learnable():
    torch.manual_seed(0)
    ds = ppe.SyntheticPPE(4, seed=0)
    x, b, l, _ = ds.detection_collate([ds[i] for i in range(4)])
    m = ppe.build_model(None, 3, TINY)
    opt = torch.optim.SGD(m.parameters(), lr=1e-2, momentum=0.9)
    x = ppe.preprocess_img(x)
    losses = []
    for _ in range(15):
        opt.zero_grad()
        loss = torch.nn.functional.binary_cross_entropy_with_logits(m(x, b), l)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0] * 0.7


def test_ppe_main_ddp_gloo(tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "ppe_main_ddp.py"), "-synthetic", "8", "-tiny", "-num_epoch", "0",
           "-batch_size", "2", "-max_iters", "1", "-backend", "gloo", "-world_size", "2", "-load_model", "none",
           "-save_model", str(tmp_path / "sm"), "-eval"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29581", PYTHONPATH=ROOT)
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.count("start training") == 2 and "mAP = " in r.stdout
    assert (tmp_path / "sm" / "model-ep0.pth").exists()


@pytest.mark.gpu
def test_ppe_train_on_gpu(tmp_path):
    from distributeddataparallel_cifar10_amd.parallel.flat_ddp import FlatBucketDDP
    dev = torch.device("cuda", 0)
    ds = ppe.SyntheticPPE(8, seed=0)
    dl = torch.utils.data.DataLoader(ds, batch_size=4, collate_fn=ds.detection_collate, drop_last=True)
    model = ppe.build_model(None, 3).to(dev)  # full ResNet-101 trunk
    tl, vl = ppe.train(dl, dl, FlatBucketDDP(model), str(tmp_path), 1, 0, device=dev)
    assert np.isfinite(tl) and np.isfinite(vl)
    mAP, *aps = ppe.eval_model(model, dl, str(tmp_path), ["rc", "nc", "ma"], dev)
    assert 0.0 <= mAP <= 1.0


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.gpu
def test_ppe_roi_ops_matches_torch():
    """ResNet101ROI on the ops layer's HIP kernels (the GPU default) vs the same weights on stock fp32 torch
    (engine='torch'): training-mode logits, loss and parameter gradients; then eval-mode (inference BN with the
    running statistics) logits.  Gradient bar: within 2x stock bf16 autocast's own error (+0.02)."""
    import copy
    from distributeddataparallel_cifar10_amd.runtime import native  # noqa: F401
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = ppe.build_model(None, 3, layers=(1, 1, 1, 1)).to(dev)
    ref = copy.deepcopy(m)
    ref.engine = "torch"
    amp = copy.deepcopy(ref)
    ds = ppe.SyntheticPPE(4, seed=0)
    imgs, boxes, labels, _ = ds.detection_collate([ds[i] for i in range(4)])
    x = ppe.preprocess_img(imgs.to(dev).float())
    b, l = boxes.to(dev).float(), labels.to(dev).float()
    out = m(x, b)
    oref = ref(x, b)
    assert out.dtype == torch.float32 and out.shape == oref.shape
    assert _rel(out.detach(), oref.detach()) < 5e-2, _rel(out.detach(), oref.detach())
    loss = torch.nn.functional.binary_cross_entropy_with_logits(out, l)
    lref = torch.nn.functional.binary_cross_entropy_with_logits(oref, l)
    loss.backward()
    lref.backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):  # stock bf16's own error on the same step sets the bar
        lamp = torch.nn.functional.binary_cross_entropy_with_logits(amp(x, b).float(), l)
    lamp.backward()
    assert abs(loss.item() - lref.item()) < 2e-2 * max(1.0, abs(lref.item()))
    for (n, p), (_, q), (_, r) in zip(m.named_parameters(), ref.named_parameters(), amp.named_parameters()):
        assert p.grad is not None, n
        assert _rel(p.grad, q.grad) <= 2 * _rel(r.grad, q.grad) + 0.02, (n, _rel(p.grad, q.grad), _rel(r.grad, q.grad))
    for a, c in zip(m.buffers(), ref.buffers()):  # BN running stats / counters updated alike
        assert torch.allclose(a.double(), c.double(), rtol=3e-2, atol=3e-2)
    m.eval()
    ref.eval()
    with torch.no_grad():
        e, eref = m(x, b), ref(x, b)
    assert _rel(e, eref) < 5e-2, _rel(e, eref)
