"""Worker for the multi-process (gloo, 127.0.0.1) tests in test_dist.py.

    python tests/_dist_worker.py <case> <out_path> [args...]

Rank/world come from RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT like torchrun.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def _init():
    dist.init_process_group("gloo", init_method="env://")
    return dist.get_rank(), dist.get_world_size()


def case_buckets(out, bucket_mb):
    """GradBucketer (hooks + async per-bucket all-reduce) == plain per-parameter all-reduce."""
    from euromillioner_amd.models.mlp import DrawMLP
    from euromillioner_amd.parallel.buckets import GradBucketer

    rank, world = _init()
    torch.manual_seed(100 + rank)
    x = torch.randn(64, 62)
    y = (torch.rand(64, 62) < 0.1).float()
    net_a = DrawMLP((62, 96, 80, 62), seed=1)
    net_b = DrawMLP((62, 96, 80, 62), seed=1)
    bk = GradBucketer(net_a, bucket_mb=float(bucket_mb), world=world)
    bk.zero_grad()
    net_a.loss(net_a(x), y).backward()
    bk.finish()
    net_b.loss(net_b(x), y).backward()
    for p in net_b.parameters():
        dist.all_reduce(p.grad)
        p.grad /= world
    err = max(float((pa.grad - pb.grad).abs().max()) for pa, pb in zip(net_a.parameters(), net_b.parameters()))
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"max_err": err, "n_buckets": len(bk.buckets)}, f)
    dist.destroy_process_group()


def case_forest(out):
    """Tree-parallel forest (C5) on `world` ranks."""
    import numpy as np

    from euromillioner_amd.data.draws import DrawSet
    from euromillioner_amd.models.forest import RandomForest, draw_features

    rank, world = _init()
    ds = DrawSet.synthetic(n=900, seed=3, planted=0.5, calendar=False)
    X, Y, F = draw_features(ds.numbers)
    rf = RandomForest(n_trees=7, max_depth=4, seed=2, device="cpu").fit(X, Y, F, group=dist.group.WORLD)
    if rank == 0:
        np.savez(out, feat=rf.feat, value=rf.value)
    dist.destroy_process_group()


def case_gbdt(out, objective="reg:logistic"):
    """Data-parallel boosting (C4): each rank fits on its row shard with all-reduced histograms."""
    import numpy as np

    from euromillioner_amd.data.draws import DrawSet
    from euromillioner_amd.models.gbdt import GBDT
    from euromillioner_amd.parallel.dist import DistInfo, shard_range
    from euromillioner_amd.pipeline import gbdt_dataset
    from euromillioner_amd import config as C

    rank, world = _init()
    ds = DrawSet.synthetic(n=700, seed=4, planted=0.6, calendar=True)
    X, Y, _ = gbdt_dataset(ds, C.RunConfig())
    Y = Y[:, :6]
    if objective.startswith("multi:"):  # class = first of the 6 numbers drawn (0 = none); rank 1 never sees 6
        Y = np.where(Y.any(1), np.argmax(Y, 1) + 1, 0).astype(np.float64)
        if rank == 1:
            Y = np.minimum(Y, 5)
    n_tr = 500
    a, b = shard_range(n_tr, DistInfo(rank, world))
    va, vb = shard_range(len(X) - n_tr, DistInfo(rank, world))
    m = GBDT(eta=0.5, max_depth=3, gamma=0.5, min_child_weight=0.5, nround=8, backend="numpy", objective=objective)
    m.fit(X[a:b], Y[a:b], evals={"test": (X[n_tr + va:n_tr + vb], Y[n_tr + va:n_tr + vb])}, group=dist.group.WORLD)
    if rank == 0:
        np.savez(out, feat=m.trees.feat, sbin=m.trees.sbin, leaf=m.trees.leaf,
                 hist=np.array([h["test"] for h in m.history]))
    dist.destroy_process_group()


if __name__ == "__main__":
    case = sys.argv[1]
    globals()["case_" + case](*sys.argv[2:])
