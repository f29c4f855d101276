"""MLP models for 62-in / 62-out draw prediction.

The north star re-implements the DL4J ``MultiLayerNetwork`` path that the reference
declares (``pom.xml:62-66``, "Neural Networks" in ``README.md:6``) but never builds.
Two execution paths share one parameter convention (DL4J layer order, per layer
``W [nIn, nOut]`` then ``b [nOut]``):

* :class:`DrawMLP` — a ``torch.nn.Module`` for arbitrary layer sizes / lag windows.
  On the GPU its dense layers run on our MFMA GEMM kernels
  (:mod:`euromillioner_amd.ops.linear`); on the CPU it is plain PyTorch (the
  world_size=1 plumbing config of BASELINE.json).
* :class:`FusedSmallMLP` — the flagship 62->128->62 trainer: one fused HIP launch for
  forward+loss+backward (``csrc/mlp_fused.hip``) plus one fused Adam launch
  (``csrc/adam.hip``), optional RCCL data parallelism in between.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn

from . import losses as L


def dl4j_xavier_(w: torch.Tensor, fan_in: int, fan_out: int, gen: torch.Generator | None = None) -> torch.Tensor:
    """DL4J ``WeightInit.XAVIER``: N(0, 2 / (nIn + nOut))."""
    with torch.no_grad():
        w.normal_(0.0, math.sqrt(2.0 / (fan_in + fan_out)), generator=gen)
    return w


class DrawMLP(nn.Module):
    def __init__(self, sizes=(62, 128, 62), activation: str = "relu", loss: str = "softmax", seed: int = 0,
                 use_hip: bool | None = None, dtype: torch.dtype = torch.float32):
        super().__init__()
        if len(sizes) < 2:
            raise ValueError("need at least input and output sizes")
        if activation not in ("relu", "sigmoid", "tanh", "identity"):
            raise ValueError(f"unknown activation {activation}")
        self.sizes = tuple(int(s) for s in sizes)
        self.activation = activation
        self.loss_name = loss
        self.use_hip = use_hip
        self.compute_dtype = dtype
        self.layers = nn.ModuleList(nn.Linear(a, b) for a, b in zip(self.sizes[:-1], self.sizes[1:]))
        g = torch.Generator().manual_seed(seed)
        for lin in self.layers:
            dl4j_xavier_(lin.weight, lin.in_features, lin.out_features, g)
            nn.init.zeros_(lin.bias)

    def _act(self, x):
        if self.activation == "relu":
            return torch.relu(x)
        if self.activation == "sigmoid":
            return torch.sigmoid(x)
        if self.activation == "tanh":
            return torch.tanh(x)
        return x

    def _hip_ok(self, x: torch.Tensor) -> bool:
        if not x.is_cuda:
            return False
        return self.use_hip is not False

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self._hip_ok(x):
            from ..ops import linear as LIN

            act = {"relu": "relu", "sigmoid": "sigmoid", "identity": "none", "tanh": "tanh"}[self.activation]
            return LIN.mlp(x, [lin.weight for lin in self.layers], [lin.bias for lin in self.layers], act)
        h = x.to(self.compute_dtype) if self.compute_dtype != torch.float32 else x
        for i, lin in enumerate(self.layers):
            w, b = lin.weight, lin.bias
            if self.compute_dtype != torch.float32:
                w, b = w.to(self.compute_dtype), b.to(self.compute_dtype)
            h = torch.nn.functional.linear(h, w, b)
            if i < len(self.layers) - 1:
                h = self._act(h)
        return h.float()

    def loss(self, logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        return L.LOSSES[self.loss_name](logits, target)

    def n_params(self) -> int:
        return sum(p.numel() for p in self.parameters())


class FusedSmallMLP:
    """Flagship trainer: 62->128->62 ReLU MLP, bf16 MFMA compute, fp32 master weights + Adam.

    Single process: two launches per optimizer step (train kernel, then ``em_adam_slab``).  A
    one-launch form (slab reduction + Adam inside the train kernel) was bit-identical but measured
    4.3 us per step slower on MI355X (93.3 vs 89.0 us, docs/DESIGN.md §6b) and was removed in round 4.
    Data parallel over xGMI: train kernel -> ``em_adam_slab_xgmi`` (two launches); over RCCL: train
    kernel -> slab reduce -> all-reduce -> Adam."""

    def __init__(self, device: str | torch.device = "cuda", loss: str = "softmax", lr: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, seed: int = 0,
                 state_dict: dict | None = None, process_group=None, comm: str = "auto",
                 dtype: str = "bf16"):
        from ..ops import fused_mlp as FM
        from ..ops import _native as N

        if loss not in FM.LOSS_KINDS:
            raise ValueError(f"loss must be one of {list(FM.LOSS_KINDS)}")
        if dtype not in ("bf16", "fp32"):
            raise ValueError("dtype must be bf16 or fp32")
        # fp32: the exact-fp32 train kernel (csrc/mlp_fused_f32.hip) on the same slabs / Adam
        self.dtype = dtype
        self.FM = FM
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("FusedSmallMLP runs on the GPU (use DrawMLP for CPU)")
        N.lib()  # fail loudly if the HIP library is missing
        self.loss_name = loss
        self.group = process_group
        dev = self.device
        P = FM.P_TOTAL
        if state_dict is None:
            ref = DrawMLP((62, 128, 62), seed=seed)
            state_dict = {"l1.weight": ref.layers[0].weight.data, "l1.bias": ref.layers[0].bias.data,
                          "l2.weight": ref.layers[1].weight.data, "l2.bias": ref.layers[1].bias.data}
        self.params = FM.flatten(state_dict, device=dev)
        self.m = torch.zeros(P, dtype=torch.float32, device=dev)
        self.v = torch.zeros(P, dtype=torch.float32, device=dev)
        self.hp = torch.tensor([lr, betas[0], betas[1], eps, weight_decay], dtype=torch.float32, device=dev)
        self.state = torch.zeros(2, dtype=torch.int32, device=dev)  # {adam step, ticket}
        self.img = torch.zeros(FM.IMG_BYTES, dtype=torch.uint8, device=dev)
        self.nslab_max = N.cu_count(dev)
        self.slabs = torch.zeros(self.nslab_max, FM.SLAB_STRIDE, dtype=torch.float32, device=dev)
        self.loss_slabs = torch.zeros(self.nslab_max, dtype=torch.float32, device=dev)
        self.grad_io = torch.zeros(P + 1, dtype=torch.float32, device=dev)  # [grads..., loss]
        self.loss_out = torch.zeros(1, dtype=torch.float32, device=dev)
        FM.pack(self.params, self.img)
        self._checked = False
        # DP gradient all-reduce: "xgmi" = one-shot peer-memory reduction fused into the Adam
        # kernel (parallel/xgmi.py), "rccl" = torch.distributed all_reduce between two Adam
        # launches; "auto" = xgmi when the node supports it (verified collectively), else rccl.
        if comm not in ("auto", "xgmi", "rccl"):
            raise ValueError("comm must be auto, xgmi or rccl")
        self.xgmi = None
        if process_group is not None and comm != "rccl":
            from ..parallel.xgmi import XgmiComm

            self.xgmi = XgmiComm.create(process_group, dev, P + 1, required=(comm == "xgmi"))
        self.comm = "xgmi" if self.xgmi is not None else ("rccl" if process_group is not None else "none")

    # ------------------------------------------------------------------ training
    @property
    def world(self) -> int:
        if self.group is None:
            return 1
        import torch.distributed as dist

        return dist.get_world_size(self.group)

    @staticmethod
    def prepare(draws) -> torch.Tensor:
        """Draw rows (numpy [N,8] or GPU uint8 [N,8]) -> device feature masks consumed by every method."""
        from ..ops import fused_mlp as FM

        if isinstance(draws, torch.Tensor):
            if draws.dtype == torch.int64 and draws.dim() == 1:
                return draws
            return FM.rows_to_masks(draws.cuda() if not draws.is_cuda else draws)
        return FM.masks_from_numpy(draws, "cuda")

    def step(self, draws: torch.Tensor, B: int, offset: int = 0, sidx: torch.Tensor | None = None,
             global_batch: int | None = None) -> torch.Tensor:
        """One optimizer step over B local samples (``draws`` = feature masks from :meth:`prepare`);
        returns the (global) mean loss as a device tensor."""
        FM = self.FM
        gb = global_batch if global_batch is not None else B * self.world
        scale = 1.0 / max(gb, 1)
        if self.loss_name == "bce":
            scale /= 62.0
        lscale = 1.0 / max(gb, 1) / (62.0 if self.loss_name == "bce" else 1.0)
        # the train kernel advances the Adam step counter (one store), so no Adam launch below draws a
        # grid-wide ticket for it (pre=True)
        nslab = self._partials(draws, B, offset, sidx, check=not self._checked, step=self.state)
        self._checked = True
        if self.group is None:
            FM.adam_slab(self.slabs, nslab, scale, self.params, self.m, self.v, self.hp, self.state, mode=0,
                         img=self.img, loss_slabs=self.loss_slabs, loss_out=self.loss_out, loss_scale=lscale, pre=True)
            return self.loss_out
        if self.xgmi is not None:  # one launch: slab reduce -> own slot, exchange, rank-order sum, Adam
            FM.adam_slab_xgmi(self.xgmi.handle, self.slabs, nslab, scale, self.params, self.m, self.v, self.hp,
                              self.state, self.loss_slabs, img=self.img, loss_out=self.loss_out, loss_scale=lscale,
                              pre=True, max_blocks=self.xgmi.consumer_blocks)
            return self.loss_out
        import torch.distributed as dist

        loss_view = self.grad_io[FM.P_TOTAL:]
        FM.adam_slab(self.slabs, nslab, scale, self.params, self.m, self.v, self.hp, self.state, mode=1,
                     grad_io=self.grad_io, loss_slabs=self.loss_slabs, loss_out=loss_view, loss_scale=lscale)
        dist.all_reduce(self.grad_io, op=dist.ReduceOp.SUM, group=self.group)
        FM.adam_slab(None, 0, 1.0, self.params, self.m, self.v, self.hp, self.state, mode=2, grad_io=self.grad_io,
                     img=self.img, pre=True)
        return loss_view

    @property
    def graph_safe(self) -> bool:
        """True when a step can be replayed from a hipGraph: single GPU, xGMI, or -- opt-in with
        ``EUROM_RCCL_GRAPH=1`` -- the RCCL path (an RCCL all-reduce is a stream-ordered kernel and
        captures like any other, so the fallback would not pay ~4 Python launches per 90 us step).
        The captured RCCL step is checked only on a 1-rank NCCL group (tests/test_train_gpu.py: replay
        == eager): RCCL refuses two ranks on one GPU, so no world >= 2 capture has run on this pool's
        1-GPU boxes, and the fallback steps eagerly until a multi-GPU node has confirmed it.  gloo
        collectives run on the host and are never captured."""
        if self.group is None or self.xgmi is not None:
            return True
        import os

        import torch.distributed as dist

        return dist.get_backend(self.group) == "nccl" and os.environ.get("EUROM_RCCL_GRAPH", "0") == "1"

    def check_comm(self) -> None:
        """Raise if an xGMI peer wait timed out (synchronises)."""
        if self.xgmi is not None:
            self.xgmi.check()

    def close(self) -> None:
        if self.xgmi is not None:
            torch.cuda.synchronize(self.device)
            self.xgmi.close()
            self.xgmi = None

    def _partials(self, draws, B, offset, sidx, check=True, step=None) -> int:
        """The train kernel of this model's dtype: per-workgroup gradient slabs; returns the grid size."""
        if self.dtype == "fp32":
            return self.FM.train_partials_f32(draws, B, self.params, self.slabs, self.loss_slabs,
                                              loss=self.loss_name, offset=offset, sidx=sidx, check=check, step=step)
        return self.FM.train_partials(draws, B, self.img, self.slabs, self.loss_slabs, loss=self.loss_name,
                                      offset=offset, sidx=sidx, check=check, step=step)

    def grads(self, draws: torch.Tensor, B: int, offset: int = 0, sidx: torch.Tensor | None = None):
        """(mean loss, flat gradient) without updating — for tests / gradient checks."""
        FM = self.FM
        nslab = self._partials(draws, B, offset, sidx)
        scale = 1.0 / B / (62.0 if self.loss_name == "bce" else 1.0)
        FM.adam_slab(self.slabs, nslab, scale, self.params, self.m, self.v, self.hp, self.state, mode=1,
                     grad_io=self.grad_io, loss_slabs=self.loss_slabs, loss_out=self.grad_io[FM.P_TOTAL:],
                     loss_scale=scale)
        g = self.grad_io[:FM.P_TOTAL].clone()
        return self.grad_io[FM.P_TOTAL].item(), g

    # ------------------------------------------------------------------ inference / eval
    def logits(self, draws: torch.Tensor, B: int, offset: int = 0, sidx=None) -> torch.Tensor:
        if self.dtype == "fp32":
            # evaluation in fp32 as well: the exact-fp32 MFMA GEMM (csrc/gemm_f32.hip) on the master
            # weights, bias + relu in its epilogue; W1 / W2 are read as [K, N] operands in place
            from ..ops import linear_f32 as LF

            FM = self.FM
            x = LF.onehot(draws, B, offset=offset, which=0, sidx=sidx)  # [B, 64], no bias column
            W1 = self.params[FM.P_W1:FM.P_W2].view(64, 128)
            W2 = self.params[FM.P_W2:FM.P_B2].view(128, 64)
            h = torch.empty(B, 128, dtype=torch.float32, device=self.device)
            LF.gemm_f32(x, True, W1, False, h, B, 128, 64, bias=W1[62], act="relu")
            z = torch.empty(B, 64, dtype=torch.float32, device=self.device)
            return LF.gemm_f32(h, True, W2, False, z, B, 64, 128, bias=self.params[FM.P_B2:FM.P_TOTAL])
        return self.FM.forward_logits(draws, B, self.img, offset=offset, sidx=sidx)

    def evaluate(self, draws: torch.Tensor, B: int, offset: int = 0, sidx=None, chunk: int = 1 << 22) -> dict:
        FM = self.FM
        tot = np.zeros(8, dtype=np.float64)
        done = 0
        while done < B:
            b = min(chunk, B - done)
            lg = self.logits(draws, b, offset=offset + done if sidx is None else 0,
                             sidx=None if sidx is None else sidx[done:done + b])
            part = FM.draw_metrics(lg, draws, b, loss=self.loss_name, offset=offset + done if sidx is None else 0,
                                   sidx=None if sidx is None else sidx[done:done + b])
            tot += part.double().sum(0).cpu().numpy()
            done += b
        if self.group is not None:
            import torch.distributed as dist

            t = torch.tensor(tot, dtype=torch.float64, device=self.device)
            dist.all_reduce(t, group=self.group)
            tot = t.cpu().numpy()
        cnt = max(tot[7], 1.0)
        out = {k: float(tot[i] / cnt) for i, k in enumerate(FM.METRIC_NAMES[:-1])}
        out["count"] = int(tot[7])
        return out

    # ------------------------------------------------------------------ state
    def state_dict(self) -> dict[str, torch.Tensor]:
        return {k: v.detach().clone().cpu() for k, v in self.FM.unflatten(self.params).items()}

    def optimizer_state(self) -> dict:
        FM = self.FM
        return {"m": {k: v.clone().cpu() for k, v in FM.unflatten(self.m).items()},
                "v": {k: v.clone().cpu() for k, v in FM.unflatten(self.v).items()},
                "step": int(self.state[0].item()),
                "hp": self.hp.cpu().tolist()}

    def load_optimizer_state(self, st: dict) -> None:
        FM = self.FM
        self.m.copy_(FM.flatten(st["m"], device=self.device))
        self.v.copy_(FM.flatten(st["v"], device=self.device))
        self.state[0] = int(st.get("step", 0))
        self.state[1] = 0

    def load_state_dict(self, sd: dict) -> None:
        self.params.copy_(self.FM.flatten(sd, device=self.device))
        self.FM.pack(self.params, self.img)

    def broadcast_parameters(self, src: int = 0) -> None:
        """C2: initial parameter sync (identical init on every rank)."""
        if self.group is None:
            return
        import torch.distributed as dist

        dist.broadcast(self.params, src=dist.get_global_rank(self.group, src) if hasattr(dist, "get_global_rank")
                       else src, group=self.group)
        self.FM.pack(self.params, self.img)
