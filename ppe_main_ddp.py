"""DDP fine-tuning of a ResNet-101 ROI multi-label classifier on PPE data (reference ``ppe_main_ddp.py``).

Same single-dash flags and defaults as the reference (``ppe_main_ddp.py:28-37``):
    python ppe_main_ddp.py -data_root integrated-above -load_model ppe_res101_professional_finished.pt \\
        -save_model saved_model [-freeze] -num_epoch 50 -target rc_nc_ma [-cv_mode]
one rank per visible GPU via ``mp.spawn``, RCCL process group, ``FlatBucketDDP`` (bucketed all-reduce overlapped
with the backward) + ``FlatSGD(lr=1e-3, momentum=0.9)``.

Extra flags (all optional): ``-ppe_root`` (the reference hard-codes ``/home/beomseok/...``), ``-synthetic N``
(offline synthetic PPE data), ``-batch_size``, ``-max_iters`` (per epoch), ``-eval`` (run eval_model after
training), ``-pre_generate OUT_DIR`` (write box-annotated predictions + JSON), ``-backend {nccl,gloo}``,
``-world_size``, ``-tiny`` (1-1-1-1 bottleneck trunk, for smoke runs).  The pieces live in
``distributeddataparallel_cifar10_amd/apps/ppe.py``.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.multiprocessing as mp

from distributeddataparallel_cifar10_amd.apps.ppe import (PPEDataset, SyntheticPPE, build_model, eval_model,
                                                           freeze_backbone, k_fold_cv, pre_generate_labels, train)
from distributeddataparallel_cifar10_amd.parallel import dist as pdist
from distributeddataparallel_cifar10_amd.parallel.flat_ddp import FlatBucketDDP

parser = argparse.ArgumentParser(description=__doc__.splitlines()[0])
parser.add_argument('-data_root', type=str, default='integrated-above',
                    choices=['above_cleaned_k=3,s=5', 'above_cleaned', 'above_all', 'integrated-complete',
                             'complete_views', 'above_view', 'integrated-above'])
parser.add_argument('-load_model', type=str, default="ppe_res101_professional_finished.pt")
parser.add_argument('-save_model', type=str, default="saved_model")
parser.add_argument('-freeze', action='store_true')
parser.add_argument('-num_epoch', type=int, default=50)
parser.add_argument('-target', type=str, default='rc_nc_ma', choices=['rc_nc_ma', 'ca_ea_ma'])
parser.add_argument('-cv_mode', action='store_true')
# additions
parser.add_argument('-ppe_root', type=str, default=os.environ.get("PPE_ROOT", "ppe_data/PPE_Profession_finished"))
parser.add_argument('-synthetic', type=int, default=0, help="use N synthetic PPE images instead of the dataset")
parser.add_argument('-batch_size', type=int, default=32)
parser.add_argument('-max_iters', type=int, default=0)
parser.add_argument('-eval', action='store_true')
parser.add_argument('-pre_generate', type=str, default="")
parser.add_argument('-backend', type=str, default="nccl", choices=["nccl", "gloo"])
parser.add_argument('-world_size', type=int, default=0)
parser.add_argument('-tiny', action='store_true')


def setup(rank, world_size, backend="nccl"):
    """Reference ppe_main_ddp.py:399-402 (127.0.0.1 instead of localhost; device bound explicitly)."""
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    pdist.setup(rank, world_size, backend=backend)


def _datasets(args):
    if args.synthetic:
        n_test = max(args.synthetic // 4, 2)
        return SyntheticPPE(args.synthetic, seed=0), SyntheticPPE(n_test, seed=1)
    base = os.path.join(args.ppe_root, args.data_root)
    return (PPEDataset(os.path.join(base, "img_train"), os.path.join(base, "label_train"), args.target),
            PPEDataset(os.path.join(base, "img_test"), os.path.join(base, "label_test"), args.target))


def main(rank, world_size, args):
    setup(rank, world_size, args.backend)
    try:
        device = torch.device("cuda", rank) if args.backend == "nccl" else torch.device("cpu")
        target_list = str(args.target).split("_")
        layers = (1, 1, 1, 1) if args.tiny else (3, 4, 23, 3)
        print("==========options provided==========")
        print('img root:', args.data_root)
        print('model load directory:', args.load_model)
        print('model save directory:', args.save_model)
        print("freeze option {}".format(args.freeze))
        print("number of epoch: {}".format(args.num_epoch))
        print("target: {}".format(args.target))
        print("cross validation option: {}".format(args.cv_mode))
        ds_train, ds_test = _datasets(args)
        print("number of train dataset: {}".format(len(ds_train)))
        print("number of test dataset: {}".format(len(ds_test)))
        if args.cv_mode:
            if rank == 0:
                k_fold_cv(ds_train, 5, args.load_model, args.save_model, args.num_epoch, target_list, args.freeze,
                          device, batch_size=args.batch_size, max_iters=args.max_iters or None, layers=layers)
            return
        tr_s = torch.utils.data.distributed.DistributedSampler(ds_train, num_replicas=world_size, rank=rank)
        te_s = torch.utils.data.distributed.DistributedSampler(ds_test, num_replicas=world_size, rank=rank)
        nw = 0 if args.synthetic else min(8, os.cpu_count() or 1)
        dl_train = torch.utils.data.DataLoader(ds_train, batch_size=args.batch_size, sampler=tr_s, num_workers=nw,
                                               collate_fn=ds_train.detection_collate, drop_last=True,
                                               pin_memory=device.type == "cuda")
        dl_test = torch.utils.data.DataLoader(ds_test, batch_size=args.batch_size, sampler=te_s, num_workers=nw,
                                              collate_fn=ds_test.detection_collate,
                                              pin_memory=device.type == "cuda")
        model = build_model(args.load_model, len(target_list), layers)
        if args.freeze:  # before the wrap, so frozen tensors stay out of the flat gradient buffer
            freeze_backbone(model)
            for name, p in model.named_parameters():
                if p.requires_grad:
                    print(f'{name} is trainable')
        model.to(device)
        ddp = FlatBucketDDP(model)
        train(dl_train, dl_test, ddp, args.save_model, args.num_epoch, rank, device=device,
              max_iters=args.max_iters or None)
        if args.eval and rank == 0:
            eval_model(model, dl_test, args.save_model, target_list, device)
        if args.pre_generate and rank == 0:
            pre_generate_labels(model, ds_test, None, out_dir=args.pre_generate,
                                json_path=os.path.join(args.pre_generate, "PPE_preds_160.json"), device=device)
    finally:
        pdist.teardown()


if __name__ == '__main__':
    args = parser.parse_args()
    if args.backend == "gloo":
        world_size = args.world_size or 1
    else:
        world_size = args.world_size or torch.cuda.device_count()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    mp.spawn(main, args=(world_size, args), nprocs=world_size)
    sys.exit(0)
