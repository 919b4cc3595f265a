"""Stage-by-stage numerical diagnostic of the fused engine against the fp32 PyTorch oracle (GPU).

Prints one line per compared tensor with the relative error max|a-b|/max|b| and a final JSON summary.
Used during development and by tests/test_engine_gpu.py.
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from model.resnet import NetResDeep  # noqa: E402
from distributeddataparallel_cifar10_amd.runtime.engine import (  # noqa: E402
    EngineConfig, NetResDeepEngine, LAYOUT)
from distributeddataparallel_cifar10_amd.utils.oracle import reference_step, nchw_to_nhwc  # noqa: E402


def rel(a: torch.Tensor, b: torch.Tensor) -> float:
    """max|a-b| / max|b|"""
    a = a.detach().double().cpu().reshape(-1)
    b = b.detach().double().cpu().reshape(-1)
    den = b.abs().max().item()
    return (a - b).abs().max().item() / (den if den > 0 else 1.0)


def rel_l2(a: torch.Tensor, b: torch.Tensor) -> float:
    """||a-b||_2 / ||b||_2 (robust to the rare ReLU-mask flips at |z| ~ 0)"""
    a = a.detach().double().cpu().reshape(-1)
    b = b.detach().double().cpu().reshape(-1)
    den = b.norm().item()
    return (a - b).norm().item() / (den if den > 0 else 1.0)


def _cfg(dtype, rows, B, persistent):
    return EngineConfig(batch_max=max(B, 32), lr=1e-2, dtype=dtype, rows=rows, persistent=persistent,
                        debug=bool(persistent))


def compare_one_step(dtype: str, rows: int, B: int, graph: bool, seed: int = 0, verbose: bool = True,
                     persistent: bool = False, forced: bool = False) -> dict:
    """One engine step vs the oracle.  forced=True feeds the engine's own stem output and conv outputs into the
    oracle (utils/oracle.py reference_step(force=...)), so the backward comparison is free of ReLU / max-pool mask
    flips and measures arithmetic error only."""
    torch.manual_seed(seed)
    dev = torch.device("cuda", 0)
    ndata = 2 * B + 8
    data = torch.randint(0, 256, (ndata, 3, 32, 32), dtype=torch.uint8)
    labels = torch.randint(0, 10, (ndata,), dtype=torch.int64)
    idx = torch.randperm(ndata)[:B]
    model = NetResDeep()
    ref = copy.deepcopy(model)
    model = model.to(dev)
    eng = NetResDeepEngine(model, data.to(dev), labels.to(dev), _cfg(dtype, rows, B, persistent))
    eng.set_indices(idx.numpy())
    eng.set_cursor(0)
    eng.read_loss(reset=True)
    eng.run(B, 1, graph=graph)
    eng.sync()
    force = None
    if forced:
        to_nchw = lambda t: t.permute(0, 3, 1, 2).contiguous().cpu()  # noqa: E731
        force = {"x0": to_nchw(eng.activations("X", 1, B)[0]),
                 "c1": eng.region("C1", B * 32 * 1024).view(B, 32, 32, 32).cpu(),
                 "y": [to_nchw(t) for t in eng.activations("Y", 10, B)]}
    r = reference_step(ref, data[idx], labels[idx], lr=1e-2, bf16_operands=(dtype == "bf16"),
                       fc1_bf16=bool(persistent) and dtype == "bf16", force=force)
    out = {}

    def rep(name, a, b):
        e, e2 = rel(a, b), rel_l2(a, b)
        out[name] = e2
        if verbose:
            print(f"  {name:28s} max_rel={e:.3e}  l2_rel={e2:.3e}", flush=True)

    loss, steps = eng.read_loss()
    rep("loss", torch.tensor([loss]), torch.tensor([r["loss"]]))
    n = B * 8192
    X = eng.activations("X", 10, B)
    Y = eng.activations("Y", 10, B)
    DY = eng.activations("DY", 10, B)
    G = eng.activations("G", 2, B)
    for i in range(10):
        rep(f"x{i}", X[i], nchw_to_nhwc(r["x"][i]))
    for i in range(10):
        rep(f"y{i}", Y[i], nchw_to_nhwc(r["y"][i]))
    for i in range(0 if persistent else 1, 10):
        rep(f"dy{i}", DY[i], nchw_to_nhwc(r["dy"][i]))
    rep("g2", G[0], nchw_to_nhwc(r["dx"][2]))
    rep("g1", G[1], nchw_to_nhwc(r["dx"][1]))
    grads = eng.grads.detach().cpu()
    for name, (off, shape) in LAYOUT.items():
        numel = 1
        for s in shape:
            numel *= s
        rep(f"grad:{name}", grads[off:off + numel].view(shape), r["grads"][name])
    sd = model.state_dict()
    for name, t in ref.state_dict().items():
        if name.startswith("resblocks.") and not name.startswith("resblocks.0."):
            continue
        if t.dtype == torch.int64:
            ok = int(sd[name].item()) == int(t.item())
            out[f"state:{name}"] = 0.0 if ok else 1.0
            if verbose:
                print(f"  state:{name:22s} engine={int(sd[name].item())} ref={int(t.item())}", flush=True)
        else:
            rep(f"state:{name}", sd[name], t)
    eng.close()
    return out


def trajectory(dtype: str, rows: int, B: int, steps: int, seed: int = 1, persistent: bool = False,
               seed_epoch=None) -> dict:
    """Multi-step loss trajectory + final params vs the oracle (graph mode).  seed_epoch: start the sliced engine's
    device epoch there (e.g. EPOCH_WRAP - 3: the steps cross the wrap); the result then also says where it ended."""
    torch.manual_seed(seed)
    dev = torch.device("cuda", 0)
    ndata = B * steps
    data = torch.randint(0, 256, (ndata, 3, 32, 32), dtype=torch.uint8)
    labels = torch.randint(0, 10, (ndata,), dtype=torch.int64)
    model = NetResDeep()
    ref = copy.deepcopy(model)
    model = model.to(dev)
    eng = NetResDeepEngine(model, data.to(dev), labels.to(dev), EngineConfig(
        batch_max=B, lr=1e-2, dtype=dtype, rows=rows, persistent=persistent))
    idx = torch.arange(ndata)
    if seed_epoch is not None:
        eng.set_epoch(int(seed_epoch))
    eng.set_indices(idx.numpy())
    eng.set_cursor(0)
    eng.read_loss(reset=True)
    losses_e, losses_r = [], []
    for s in range(steps):
        eng.run(B, 1, graph=True)
        lsum, _ = eng.read_loss(reset=True)
        losses_e.append(lsum)
        sel = idx[s * B:(s + 1) * B]
        losses_r.append(reference_step(ref, data[sel], labels[sel], bf16_operands=(dtype == "bf16"),
                                       fc1_bf16=bool(persistent) and dtype == "bf16")["loss"])
    sd, rsd = model.state_dict(), ref.state_dict()
    keys = [k for k in rsd if rsd[k].dtype != torch.int64]
    perr = max(rel(sd[k], rsd[k]) for k in keys)
    a = torch.cat([sd[k].detach().double().cpu().reshape(-1) for k in keys])
    b = torch.cat([rsd[k].detach().double().reshape(-1) for k in keys])
    epoch_end = eng.epoch() if persistent else None
    eng.close()
    return {"losses_engine": losses_e, "losses_ref": losses_r, "max_param_rel_err": perr,
            "param_rel_l2": ((a - b).norm() / b.norm()).item(), "params": a, "epoch_end": epoch_end}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtypes", default="fp32,bf16")
    ap.add_argument("--rows", default="4,2")
    ap.add_argument("--batches", default="32,16")
    ap.add_argument("--traj-steps", type=int, default=5)
    ap.add_argument("--persistent", type=int, default=-1, help="1: persistent engine only, 0: multi-kernel only")
    a = ap.parse_args()
    summary = {}
    if a.persistent != 0:
        for B in [int(x) for x in a.batches.split(",")]:
            for graph in (False, True):
                key = f"bf16/persistent/B{B}/{'graph' if graph else 'eager'}"
                print(f"== {key}", flush=True)
                try:
                    res = compare_one_step("bf16", 4, B, graph, persistent=True)
                    summary[key] = max(res.values())
                except Exception as exc:
                    print(f"  FAILED: {exc!r}", flush=True)
                    summary[key] = f"error: {exc}"
        print("== trajectory bf16/persistent", flush=True)
        try:
            tr = trajectory("bf16", 4, 32, a.traj_steps, persistent=True)
            print("  " + json.dumps(tr), flush=True)
            summary["traj/bf16/persistent"] = tr["max_param_rel_err"]
        except Exception as exc:
            print(f"  FAILED: {exc!r}", flush=True)
    if a.persistent == 1:
        print(json.dumps({"summary": summary}), flush=True)
        return
    for dtype in a.dtypes.split(","):
        for rows in [int(x) for x in a.rows.split(",")]:
            for B in [int(x) for x in a.batches.split(",")]:
                for graph in (False, True):
                    key = f"{dtype}/R{rows}/B{B}/{'graph' if graph else 'eager'}"
                    print(f"== {key}", flush=True)
                    try:
                        res = compare_one_step(dtype, rows, B, graph)
                        summary[key] = max(res.values())
                    except Exception as exc:  # report and continue with other configs
                        print(f"  FAILED: {exc!r}", flush=True)
                        summary[key] = f"error: {exc}"
            print(f"== trajectory {dtype}/R{rows}", flush=True)
            try:
                tr = trajectory(dtype, rows, 32, a.traj_steps)
                print("  " + json.dumps(tr), flush=True)
                summary[f"traj/{dtype}/R{rows}"] = tr["max_param_rel_err"]
            except Exception as exc:
                print(f"  FAILED: {exc!r}", flush=True)
    print(json.dumps({"summary": summary}), flush=True)


if __name__ == "__main__":
    main()
