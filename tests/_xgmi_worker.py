"""One rank of the xGMI communicator GPU test (tests/test_xgmi_gpu.py).

Rank r runs on cuda:(r % device_count): distinct GPUs (real xGMI peers) on a node with >= world
GPUs, all on cuda:0 on a 1-GPU box (IPC between processes on one device exercises the same
flag/slot protocol).  With EUROM_XGMI=0 it checks the RCCL/host fallback instead.  A gloo
group carries the handle exchange and the reference results.  Prints one JSON line.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def fallback(rank, world, dev):
    """EUROM_XGMI=0, or more than two ranks per device (XGMI_CROWDED=1): the communicator declines
    collectively, comm="xgmi" raises, and comm="auto" runs the host all-reduce."""
    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.mlp import FusedSmallMLP
    from euromillioner_amd.parallel.xgmi import XgmiComm, XgmiError

    out = {"rank": rank, "create": XgmiComm.create(dist.group.WORLD, dev, 1024) is None}
    try:
        XgmiComm.create(dist.group.WORLD, dev, 1024, required=True)
        out["required_raises"] = False
    except XgmiError as e:
        out["required_raises"] = True
        out["reason"] = str(e)
    m = FusedSmallMLP(dev, loss="softmax", lr=3e-3, seed=0, process_group=dist.group.WORLD, comm="auto")
    m.broadcast_parameters()
    out["comm"] = m.comm
    B = 4096
    draws = generate_masks(world * B + 16, seed=5, planted=0.8, device=dev)
    losses = [float(m.step(draws, B, offset=rank * B).item()) for _ in range(3)]
    torch.cuda.synchronize()
    out["finite"] = all(x == x and x > 0 for x in losses)
    allp = [torch.empty_like(m.params.cpu()) for _ in range(world)]
    dist.all_gather(allp, m.params.cpu())
    out["params_bit_identical"] = all(torch.equal(allp[0], a) for a in allp)
    m.close()
    print("XGMI_RESULT " + json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", rank % ndev)  # distinct devices whenever the node has >= world GPUs
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    if os.environ.get("EUROM_XGMI", "1") == "0" or os.environ.get("XGMI_CROWDED") == "1":
        return fallback(rank, world, dev)
    from euromillioner_amd.data.synthetic import generate_draws
    from euromillioner_amd.models.mlp import FusedSmallMLP
    from euromillioner_amd.parallel.xgmi import XgmiComm, XgmiError

    out = {"rank": rank}
    comm = XgmiComm.create(dist.group.WORLD, dev, 40000, timeout_s=20.0, required=True)
    out["cap"] = comm.cap

    # 1. generic all-reduce vs gloo, several rounds (both slots, seq wrap of the parity)
    g = torch.Generator().manual_seed(100 + rank)
    errs, same = [], True
    for rnd in range(5):
        n = [1, 257, 16449, 40000, 3][rnd]
        x = torch.randn(n, generator=g)
        ref = x.clone()
        dist.all_reduce(ref)
        y = x.to(dev)
        comm.all_reduce_(y, scale=0.5)
        torch.cuda.synchronize()
        errs.append(float((y.cpu() - 0.5 * ref).abs().max()))
        allv = [torch.empty_like(y.cpu()) for _ in range(world)]
        dist.all_gather(allv, y.cpu())
        same = same and all(torch.equal(allv[0], a) for a in allv)
    out["allreduce_err"] = max(errs)
    out["allreduce_bit_identical"] = same
    comm.check()
    comm.close()

    # 2. fused MLP DP step: xgmi vs host all-reduce (gloo here), eager and hipGraph
    nums, _ = generate_draws(40001, seed=7 + rank, planted=0.8, native=True)
    B = 8192
    models = {}
    for kind in ("xgmi", "rccl"):
        m = FusedSmallMLP(dev, loss="softmax", lr=3e-3, seed=0, process_group=dist.group.WORLD, comm=kind)
        m.broadcast_parameters()
        models[kind] = m
    assert models["xgmi"].comm == "xgmi" and models["rccl"].comm == "rccl"
    draws = FusedSmallMLP.prepare(nums)
    losses = {"xgmi": [], "rccl": []}
    for i in range(4):
        for kind, m in models.items():
            losses[kind].append(float(m.step(draws, B, offset=i * B).item()))
    torch.cuda.synchronize()
    out["loss_xgmi"], out["loss_rccl"] = losses["xgmi"], losses["rccl"]
    out["param_diff"] = float((models["xgmi"].params - models["rccl"].params).abs().max())
    # graph capture of the xgmi step (3 kernels, no host collective) == eager continuation
    mx = models["xgmi"]
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    p_before = mx.params.clone()
    m_snap, v_snap, s_snap = mx.m.clone(), mx.v.clone(), mx.state.clone()
    with torch.cuda.stream(st):
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=st):
            mx.step(draws, B, offset=0)
    torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    assert torch.equal(p_before, mx.params), "capture must not execute"
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    p_graph = mx.params.clone()
    mx.params.copy_(p_before), mx.m.copy_(m_snap), mx.v.copy_(v_snap), mx.state.copy_(s_snap)
    mx.FM.pack(mx.params, mx.img)
    for _ in range(3):
        mx.step(draws, B, offset=0)
    torch.cuda.synchronize()
    out["graph_vs_eager"] = float((p_graph - mx.params).abs().max())
    allp = [torch.empty_like(mx.params.cpu()) for _ in range(world)]
    dist.all_gather(allp, mx.params.cpu())
    out["params_bit_identical"] = all(torch.equal(allp[0], a) for a in allp)
    mx.check_comm()
    for m in models.values():
        m.close()

    # 3. timeout: rank 0 reduces while nobody else publishes -> error word, no hang
    comm = XgmiComm.create(dist.group.WORLD, dev, 256, timeout_s=2.0, required=True)
    raised = None
    if rank == 0:
        comm.stage(torch.ones(256, device=dev))
        comm.stage(torch.ones(256, device=dev))  # (same slot twice: peers never produce)
        # peers' flags never reach this seq: bounded wait
        y = torch.ones(256, device=dev)
        comm.reduce(y)
        torch.cuda.synchronize()
        try:
            comm.check()
            raised = False
        except XgmiError:
            raised = True
    dist.barrier()
    out["timeout_raised"] = raised
    comm.close()
    print("XGMI_RESULT " + json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
