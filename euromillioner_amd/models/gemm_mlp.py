"""GEMM-path MLP trainer: any ``62 -> h1 -> ... -> 62`` stack on the K1-K3 MFMA GEMM.

Used for the BASELINE "Wide MLP (62->8192->8192->62) bf16 DP=8" config and for custom
layer sizes; the 62->128->62 flagship uses the single-launch fused kernel instead
(:class:`~euromillioner_amd.models.mlp.FusedSmallMLP`).  The reference's DL4J
``MultiLayerNetwork.fit`` (declared ``pom.xml:62-66``, never called) is the behaviour
being re-implemented: dense layers, ReLU, softmax/BCE output, Adam.

Per step (all on the current HIP stream, no host sync):

1. K14 multi-hot encode of the batch straight from the 64-bit draw masks -> bf16 [B, 64];
2. forward GEMMs with fused bias+act (bf16 activations), fp32 logits;
3. K10 fused loss + dL/dlogits (bf16, pre-scaled by 1 / global batch);
4. backward, last layer first: wgrad (fp32, written in place into the flat gradient
   buffer) + bias colsum, then dgrad with act' fused.  Data parallel: a hidden layer's
   256-tile weight gradient is computed in row panels of about ``bucket_mb`` each, and each
   panel's all-reduce is launched as soon as the panel is written (``async_op``: RCCL's stream
   runs it under the next panels and the layer's dgrad GEMM), so the 8192x8192 layer's
   268 MB of fp32 gradient (~99 % of the bytes) is not held back to the end of its wgrad;
   ``comm_dtype="bf16"`` all-reduces bf16 copies of the buckets (half the xGMI bytes) and Adam
   widens them back to fp32;
5. one fused Adam over the flat fp32 master weights that also refreshes the bf16
   shadow the GEMMs read (no per-step weight casts).

Flat layout per layer (padded: input and output 62 -> 64, hidden to multiples of 8, or of 256 for
wide relu/tanh bf16 layers so they stay on the 256-tile GEMM path; the pads stay exactly zero): ``W [N_pad, K_pad]`` (nn.Linear orientation) then ``b [N_pad]``;
one extra slot at the end carries the step loss through the same all-reduce.

``dtype="fp32"`` (``--dtype fp32``) runs the same step in fp32 end to end on the exact-fp32 MFMA
GEMM (``csrc/gemm_f32.hip``): fp32 activations and dL/dZ, no bf16 shadow.

``lags=k`` (``--lags k``) takes the lag window of ``data/draws.lag_features``: the input
of sample i is the multi-hot of draws i .. i+k-1 (built on the device, K14 ``onehot_lags``; each 62-wide
block padded to 64), the target is draw i+k.  Layer 0 is then ``W [N_pad, 64k]``; the logical
``[N, 62k]`` weight maps block j's columns 62j..62j+61 to 64j..64j+61.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..ops import fused_mlp as FM
from ..ops import linear as LIN
from ..ops import linear_f32 as LF
from ..ops import _native as N
from .mlp import DrawMLP, FusedSmallMLP


def _pad(n: int) -> int:
    return (n + 7) // 8 * 8


def _pad_hidden(n: int, activation: str, dtype: str) -> int:
    """Hidden width in the flat layout.  Wide bf16 layers round up to the 256x256 GEMM tile, so every
    GEMM of the layer takes the NT / ping-pong path (~1.3 PF/s) instead of the any-shape 128x128
    fallback (0.3-0.7 PF/s measured): 1000 -> 1024 costs 2.4 % more FLOPs for ~2x the rate.  Only
    for activations with act(0) = 0 (relu, tanh), so the extra units stay exactly zero."""
    if dtype == "bf16" and activation in ("relu", "tanh") and n >= 768:
        return (n + 255) // 256 * 256
    return _pad(n)


class GemmMLPTrainer:
    def __init__(self, sizes=(62, 8192, 8192, 62), device="cuda", activation: str = "relu", loss: str = "softmax",
                 lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, seed: int = 0,
                 state_dict: dict | None = None, process_group=None, bucket_mb: float = 25.0, dtype: str = "bf16",
                 lags: int = 1, comm_dtype: str = "fp32"):
        if lags < 1 or sizes[0] != 62 * lags or sizes[-1] != 62:
            raise ValueError(f"draw MLPs are (62 * lags)-in / 62-out (lags={lags}, sizes={tuple(sizes)})")
        self.lags = int(lags)
        if activation not in ("relu", "tanh", "sigmoid"):
            raise ValueError("activation must be relu|tanh|sigmoid")
        if activation == "sigmoid" and any(h % 8 for h in sizes[1:-1]):
            raise ValueError("sigmoid needs hidden sizes that are multiples of 8 (sigmoid(0) != 0 on pads)")
        if loss not in FM.LOSS_KINDS:
            raise ValueError(f"loss must be one of {list(FM.LOSS_KINDS)}")
        if dtype not in ("bf16", "fp32"):
            raise ValueError("dtype must be bf16 or fp32")
        if comm_dtype not in ("fp32", "bf16"):
            raise ValueError("comm_dtype must be fp32 or bf16")
        self.dtype = dtype
        self.f32 = dtype == "fp32"
        self.comm_dtype = comm_dtype
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("GemmMLPTrainer runs on the GPU (use DrawMLP on the CPU)")
        N.lib()
        self.sizes = tuple(int(s) for s in sizes)
        self.padded = (64 * self.lags,) + tuple(_pad_hidden(h, activation, dtype) for h in self.sizes[1:-1]) + (64,)
        self.activation, self.loss_name, self.group = activation, loss, process_group
        # whole multiples of 8 elements: every bucket of the bf16 wire then starts 32-B aligned (the
        # fp32 -> bf16 cast takes 16-B aligned fp32 sources; flat ranges start at multiples of 8)
        self.bucket_elems = max(1 << 16, int(bucket_mb * (1 << 20) // 4) // 8 * 8)
        self.offsets = []
        off = 0
        for kp, np_ in zip(self.padded[:-1], self.padded[1:]):
            self.offsets.append((off, off + np_ * kp, off + np_ * kp + np_))
            off += np_ * kp + np_
        self.P = off
        dev = self.device
        self.params = torch.zeros(self.P, dtype=torch.float32, device=dev)
        self.grads = torch.zeros(self.P + 1, dtype=torch.float32, device=dev)
        self.m = torch.zeros(self.P, dtype=torch.float32, device=dev)
        self.v = torch.zeros(self.P, dtype=torch.float32, device=dev)
        # bf16 copy of the weights the bf16 GEMMs read (refreshed by the fused Adam); fp32 reads params
        self.shadow = None if self.f32 else torch.zeros(self.P, dtype=torch.bfloat16, device=dev)
        # bf16 wire format of the gradient (comm_dtype="bf16", data parallel only)
        self.grads_bf16 = (torch.zeros(self.P, dtype=torch.bfloat16, device=dev)
                           if comm_dtype == "bf16" and process_group is not None else None)
        self.hp = torch.tensor([lr, betas[0], betas[1], eps, weight_decay], dtype=torch.float32, device=dev)
        self.state = torch.zeros(2, dtype=torch.int32, device=dev)
        if state_dict is None:
            state_dict = DrawMLP(self.sizes, activation=activation, seed=seed).state_dict()
        self.load_state_dict(state_dict)
        self._ws_cache: dict[int, dict] = {}
        self._checked = False
        self.panel_ncu: int | None = None  # (tests: pretend a smaller GPU to get several wgrad panels)
        # (tools/wide_overlap.py: a factory (flat, bucket_elems) -> object with ready(a, c) / wait() that
        # stands in for the all-reduce on one GPU, e.g. a side-stream reduce-copy per bucket)
        self.comm_emulator = None
        self.last_buckets: list[tuple[int, int]] = []


    # ------------------------------------------------------------------ layout
    def _views(self, flat: torch.Tensor, i: int):
        a, b, c = self.offsets[i]
        np_, kp = self.padded[i + 1], self.padded[i]
        return flat[a:b].view(np_, kp), flat[b:c]

    @property
    def world(self) -> int:
        if self.group is None:
            return 1
        import torch.distributed as dist

        return dist.get_world_size(self.group)

    def flops_per_sample(self) -> float:
        """Executed MFMA FLOPs per sample (forward + wgrad + dgrad of layers >= 1), padded shapes."""
        f = 0.0
        for i, (kp, np_) in enumerate(zip(self.padded[:-1], self.padded[1:])):
            f += 2 * kp * np_ * (3 if i > 0 else 2)
        return f

    def _plan(self, B: int) -> dict:
        """Which layers run the 256-tile NT path for their weight gradient (needs transposed
        copies of dZ_i and X_i, produced by the neighbouring GEMMs' transposed epilogue)."""
        P, L = self.padded, len(self.offsets)
        big_wgrad = [False] * L
        for i in range(1, L - 1):
            big_wgrad[i] = (LIN.big_ok(P[i + 1], P[i], B) and LIN.big_ok(B, P[i + 1], P[i + 2])
                            and LIN.big_ok(B, P[i], P[i - 1]))
        big_dgrad = [i > 0 and LIN.big_ok(B, P[i], P[i + 1]) for i in range(L)]
        return {"wgrad": big_wgrad, "dgrad": big_dgrad}

    def _use_bits(self, plan: dict, B: int, i: int) -> bool:
        """X_i's act' as activity bits: relu, both GEMMs on the 256-tile paths (EUROM_RELU_BITS=0: off)."""
        import os

        P = self.padded
        return (self.activation == "relu" and plan["dgrad"][i] and B % 32 == 0
                and LIN.big_ok(B, P[i], P[i - 1]) and os.environ.get("EUROM_RELU_BITS", "1") != "0")

    def _ws(self, B: int) -> dict:
        ws = self._ws_cache.get(B)
        if ws is None and self.f32:
            dev, P = self.device, self.padded
            f = torch.float32
            ws = {"x": torch.empty(B, 64 * self.lags, dtype=f, device=dev),
                  "act": [torch.empty(B, n, dtype=f, device=dev) for n in P[1:-1]],
                  "dz": [torch.empty(B, n, dtype=f, device=dev) for n in P[1:]],
                  "logits": torch.empty(B, 64, dtype=f, device=dev),
                  "part": torch.empty(max((B + 3) // 4, 1), dtype=f, device=dev),
                  # bias-gradient partials: of dz_last from the loss kernel, of dz_{i-1} from the dgrad epilogue
                  "losscol": torch.empty(max(1, LIN.loss_grad_blocks(B)) * 64, dtype=f, device=dev),
                  "colpart": torch.empty(max(1, -(-B // 128)) * max(P), dtype=f, device=dev),
                  "parts": {}}
            self._ws_cache = {B: ws}
        if ws is None:
            dev = self.device
            plan = self._plan(B)
            L = len(self.offsets)
            P = self.padded
            ws = {"x": torch.empty(B, 64 * self.lags, dtype=torch.bfloat16, device=dev),
                  "act": [torch.empty(B, n, dtype=torch.bfloat16, device=dev) for n in P[1:-1]],
                  "dz": [torch.empty(B, n, dtype=torch.bfloat16, device=dev) for n in P[1:]],
                  "logits": torch.empty(B, 64, dtype=torch.float32, device=dev),
                  "part": torch.empty(max((B + 3) // 4, 1), dtype=torch.float32, device=dev),
                  "losscol": torch.empty(max(1, LIN.loss_grad_blocks(B)) * 64, dtype=torch.float32, device=dev),
                  "colsum_ws": torch.empty(max(1, (B + 511) // 512) * max(P), dtype=torch.float32, device=dev),
                  # bias-gradient partials [B / 128][N] written by the 256-tile dgrad epilogue (fused K3 bias grad)
                  "colpart": torch.empty(max(1, B // 128) * max(P), dtype=torch.float32, device=dev),
                  "plan": plan,
                  # transposed copies for the big wgrads: X_i^T (= Y_{i-1}^T) and dZ_i^T
                  "actt": {i: torch.empty(P[i], B, dtype=torch.bfloat16, device=dev)
                           for i in range(L) if plan["wgrad"][i]},
                  "dzt": {i: torch.empty(P[i + 1], B, dtype=torch.bfloat16, device=dev)
                          for i in range(L) if plan["wgrad"][i]},
                  "wt": {i: torch.empty(P[i], P[i + 1], dtype=torch.bfloat16, device=dev)
                         for i in range(L) if plan["dgrad"][i]},
                  # relu activity bits of X_i (written by layer i - 1's forward, read by layer i's dgrad
                  # instead of the bf16 X_i: 64x fewer bytes in the act' epilogue)
                  "bits": {i: LIN.relu_bits(B, P[i], dev) for i in range(1, L) if self._use_bits(plan, B, i)}}
            self._ws_cache = {B: ws}  # keep one batch size resident
        return ws

    # ------------------------------------------------------------------ compute
    @staticmethod
    def prepare(draws) -> torch.Tensor:
        return FusedSmallMLP.prepare(draws)

    def _tmasks(self, masks: torch.Tensor) -> torch.Tensor:
        """Masks as the loss/metric kernels see them: their target masks[i + 1] is draw i + lags."""
        return masks[self.lags - 1:] if self.lags > 1 else masks

    def _forward(self, masks, B, offset, sidx, ws, train: bool = False):
        if self.f32:
            if self.lags > 1:
                h = FM.onehot_lags(masks, B, self.lags, offset=offset, sidx=sidx, out=ws["x"], dtype=torch.float32)
            else:
                h = LF.onehot(masks, B, offset=offset, which=0, sidx=sidx, out=ws["x"])
            inputs = []
            L = len(self.offsets)
            for i in range(L):
                w, bf = self._views(self.params, i)
                inputs.append(h)
                last = i == L - 1
                h = LF.linear_fwd(h, w, bf, "none" if last else self.activation,
                                  out=ws["logits"] if last else ws["act"][i])
            return h, inputs
        if self.lags > 1:
            x = FM.onehot_lags(masks, B, self.lags, offset=offset, sidx=sidx, out=ws["x"])
        else:
            x = FM.onehot(masks, B, offset=offset, which=0, bias=False, sidx=sidx, out=ws["x"])
        h, inputs = x, []
        L = len(self.offsets)
        for i in range(L):
            w, b = self._views(self.shadow, i)
            _, bf = self._views(self.params, i)
            inputs.append(h)
            last = i == L - 1
            out = ws["logits"] if last else ws["act"][i]
            ct = ws["actt"].get(i + 1) if train and not last else None  # X_{i+1}^T for layer i+1's wgrad
            bits = ws["bits"].get(i + 1) if train and not last else None
            h = LIN.linear_fwd(h, w, bf, "none" if last else self.activation, out=out, ct=ct, bits=bits)
        return h, inputs

    def wgrad_panels(self, i: int) -> list[tuple[int, int]]:
        """Row panels of layer i's weight gradient, each all-reduced as soon as it is written
        (``parallel.buckets.plan_panels``: whole waves of 256x256 tiles, >= ``bucket_mb``)."""
        from ..parallel.buckets import plan_panels

        ncu = self.panel_ncu or N.cu_count(self.device)
        return plan_panels(self.padded[i + 1], self.padded[i], self.bucket_elems, ncu, LIN.BIG_M, LIN.BIG_N)

    def _loss_bias(self, ws, B: int, accumulate: bool) -> None:
        """Last layer's bias gradient from the loss kernel's per-block column partials."""
        _, gbias = self._views(self.grads, len(self.offsets) - 1)
        LIN.colpart_reduce(ws["losscol"], LIN.loss_grad_blocks(B), 64, gbias, accumulate=accumulate)

    def _backward(self, dz, inputs, ws, on_ready=None, accumulate: bool = False):
        """Last layer first: wgrad + bias grad into the flat gradient buffer (added to it when
        ``accumulate``: gradient accumulation over micro-batches), then dgrad (act' fused).
        ``on_ready(a, c)`` is called as soon as flat gradient range [a, c) is final: per row panel
        of a 256-tile wgrad, per whole weight otherwise, then per bias.  The last layer's bias
        gradient is already in place (``_loss_bias``); every other bias gradient comes from the
        partial column sums of the dgrad that produced its dZ."""
        L = len(self.offsets)
        if self.f32 and accumulate:
            raise ValueError("gradient accumulation runs on the bf16 path")
        B = dz.shape[0]
        if self.f32:
            for i in reversed(range(L)):
                gw, gbias = self._views(self.grads, i)
                LF.linear_wgrad(dz, inputs[i], out=gw, parts_cache=ws["parts"])
                if on_ready is not None:
                    on_ready(self.offsets[i][0], self.offsets[i][2])
                if i > 0:
                    w, _ = self._views(self.params, i)
                    dz = LF.linear_dgrad(dz, w, inputs[i], self.activation, out=ws["dz"][i - 1],
                                         colpart=ws["colpart"])
                    _, gb_prev = self._views(self.grads, i - 1)
                    LIN.colpart_reduce(ws["colpart"], -(-B // 128), self.padded[i], gb_prev)
            return dz
        plan = ws["plan"]
        fused_bias = {L - 1}  # layers whose bias gradient is already summed (loss kernel / a dgrad epilogue)
        for i in reversed(range(L)):
            gw, gbias = self._views(self.grads, i)
            beta = 1.0 if accumulate else 0.0
            a, b_off, c = self.offsets[i]
            K = self.padded[i]
            # (a big layer's dgrad on a side stream beside its wgrad -- the two GEMMs' workgroups interleaved
            # on the CUs -- measured 20.8-21.0 vs 18.8-18.9 ms per wide step, round 6: their L2 tile groups
            # and XCD placement fight; one stream)
            if plan["wgrad"][i]:
                panels = self.wgrad_panels(i) if on_ready is not None else [(0, gw.shape[0])]
                for r0, r1 in panels:  # each panel's all-reduce starts while the next panels run
                    LIN.linear_wgrad_nt(ws["dzt"][i][r0:r1], ws["actt"][i], out=gw[r0:r1], beta=beta)
                    if on_ready is not None:
                        on_ready(a + r0 * K, a + r1 * K)
                if i not in fused_bias:
                    LIN.rowsum(ws["dzt"][i], out=gbias, accumulate=accumulate)
            else:
                LIN.linear_wgrad(dz, inputs[i], out=gw, beta=beta)
                if on_ready is not None:
                    on_ready(a, b_off)
                if i not in fused_bias:
                    LIN.colsum(dz, out=gbias, accumulate=accumulate, ws=ws["colsum_ws"])
            if on_ready is not None:
                on_ready(b_off, c)
            if i > 0:
                if plan["dgrad"][i]:
                    dz = self._dgrad_big(i, dz, inputs, ws, accumulate, fused_bias)
                else:
                    w, _ = self._views(self.shadow, i)
                    dz = LIN.linear_dgrad(dz, w, inputs[i], self.activation, out=ws["dz"][i - 1])
        return dz

    def _dgrad_big(self, i, dz, inputs, ws, accumulate, fused_bias):
        """dZ_{i-1} of a big layer: the NT dgrad on W_i^T with act' from the relu bits, the K3 bias gradient
        of layer i - 1 fused into its epilogue (per-128-row column sums of dZ_{i-1}, fp32, before the bf16
        store) and one fixed-order reduce of them."""
        B = dz.shape[0]
        w, _ = self._views(self.shadow, i)
        wt = LIN.transpose(w, out=ws["wt"][i])
        part = ws["colpart"] if B % 128 == 0 else None
        dz = LIN.linear_dgrad_nt(dz, wt, inputs[i], self.activation, out=ws["dz"][i - 1],
                                 ct=ws["dzt"].get(i - 1), colpart=part, bits=ws["bits"].get(i))
        if part is not None:
            _, gb_prev = self._views(self.grads, i - 1)
            LIN.colpart_reduce(part, B // 128, self.padded[i], gb_prev, accumulate=accumulate)
            fused_bias.add(i - 1)
        return dz


    def _check(self, masks, B, offset, sidx):
        if not self._checked:
            FM._check_draws(self._tmasks(masks), sidx, B, offset)
            self._checked = True

    def step(self, masks: torch.Tensor, B: int, offset: int = 0, sidx: torch.Tensor | None = None,
             global_batch: int | None = None, accum: int = 1) -> torch.Tensor:
        """One optimizer step on ``accum`` consecutive micro-batches of B local samples (gradient
        accumulation: the mega-batch B * accum never has to fit as activations); returns the global
        mean loss (device tensor)."""
        if accum < 1 or (accum > 1 and sidx is not None):
            raise ValueError("accum >= 1, and accumulation walks consecutive samples (no sample_idx)")
        self._check(masks, B * accum, offset, sidx)
        ws = self._ws(B)
        gb = global_batch if global_batch is not None else B * accum * self.world
        for k in range(accum - 1):  # all but the last micro-batch: local accumulation only
            off = offset + k * B
            logits, inputs = self._forward(masks, B, off, None, ws, train=True)
            dz, part = LIN.loss_grad(logits, self._tmasks(masks), B, self.loss_name, offset=off, grad_scale=1.0 / gb,
                                     dz=ws["dz"][-1], partials=ws["part"], colpart=ws["losscol"])
            self._loss_bias(ws, B, accumulate=k > 0)
            if k == 0:
                torch.sum(part, dim=0, keepdim=True, out=self.grads[self.P:])
            else:
                self.grads[self.P:] += part.sum()
            self._backward(dz, inputs, ws, accumulate=k > 0)
        last = offset + (accum - 1) * B
        logits, inputs = self._forward(masks, B, last, sidx, ws, train=True)
        dz, part = (LF if self.f32 else LIN).loss_grad(logits, self._tmasks(masks), B, self.loss_name, offset=last,
                                                       sidx=sidx, grad_scale=1.0 / gb, dz=ws["dz"][-1],
                                                       partials=ws["part"], colpart=ws["losscol"])
        self._loss_bias(ws, B, accumulate=accum > 1)
        if accum == 1:
            torch.sum(part, dim=0, keepdim=True, out=self.grads[self.P:])
        else:
            self.grads[self.P:] += part.sum()
        self.grads[self.P:].mul_(1.0 / gb)
        red = None
        if self.comm_emulator is not None and self.group is None:
            red = self.comm_emulator(self.grads, self.bucket_elems)
        elif self.group is not None:
            import torch.distributed as dist

            from ..parallel.buckets import RangeAllReducer

            red = RangeAllReducer(self.grads, self.bucket_elems, self.group, wire=self.grads_bf16, cast=FM.cast_bf16)
            # the loss slot travels in fp32 on its own (tiny), before the backward starts
            red.handles.append(dist.all_reduce(self.grads[self.P:], op=dist.ReduceOp.SUM, group=self.group,
                                               async_op=True))
        self._backward(dz, inputs, ws, red.ready if red is not None else None, accumulate=accum > 1)
        if red is not None:
            red.wait()
            self.last_buckets = list(red.launched)
        g = self.grads_bf16 if self.grads_bf16 is not None else self.grads[:self.P]
        FM.adam_flat(self.params, g, self.m, self.v, self.hp, self.state, 1.0, shadow=self.shadow)
        return self.grads[self.P:]

    def grads_only(self, masks, B, offset=0, sidx=None):
        """(loss, {name: grad}) for tests: same kernels, no all-reduce, no update."""
        ws = self._ws(B)
        logits, inputs = self._forward(masks, B, offset, sidx, ws, train=True)
        dz, part = (LF if self.f32 else LIN).loss_grad(logits, self._tmasks(masks), B, self.loss_name, offset=offset,
                                                       sidx=sidx, grad_scale=1.0 / B, dz=ws["dz"][-1],
                                                       partials=ws["part"], colpart=ws["losscol"])
        self._loss_bias(ws, B, accumulate=False)
        self._backward(dz, inputs, ws)
        out = {k: v.clone() for k, v in self._logical(self.grads, flat_layer0=True).items()}
        return float(part.double().sum().item()) / B, out

    def logits(self, masks, B, offset=0, sidx=None) -> torch.Tensor:
        lg, _ = self._forward(masks, B, offset, sidx, self._ws(B))
        return lg

    def evaluate(self, masks, B, offset=0, sidx=None, chunk: int = 1 << 16) -> dict:
        tot = np.zeros(8, dtype=np.float64)
        done = 0
        while done < B:
            b = min(chunk, B - done)
            o = offset + done if sidx is None else 0
            si = None if sidx is None else sidx[done:done + b]
            lg = self.logits(masks, b, o, si)
            tot += FM.draw_metrics(lg, self._tmasks(masks), b, loss=self.loss_name, offset=o,
                                   sidx=si).double().sum(0).cpu().numpy()
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
    def _logical(self, flat: torch.Tensor, flat_layer0: bool = False) -> dict[str, torch.Tensor]:
        """Views of the logical weights.  Layer 0's weight is the view [N, lags, 62] of its padded
        [N_pad, 64 * lags] block (``flat_layer0``: a [N, 62 * lags] copy instead)."""
        out = {}
        for i in range(len(self.offsets)):
            w, b = self._views(flat, i)
            k, n = self.sizes[i], self.sizes[i + 1]
            if i == 0:
                w3 = w.view(w.shape[0], self.lags, 64)[:n, :, :62]
                out["layers.0.weight"] = w3.reshape(n, k) if flat_layer0 else w3
            else:
                out[f"layers.{i}.weight"] = w[:n, :k]
            out[f"layers.{i}.bias"] = b[:n]
        return out

    def _to_logical(self, name: str, v: torch.Tensor) -> torch.Tensor:
        return v.reshape(v.shape[0], -1) if name == "layers.0.weight" else v

    def _load_logical(self, flat: torch.Tensor, named: dict) -> None:
        for k, v in self._logical(flat).items():
            src = named[k].to(self.device, torch.float32)
            v.copy_(src.view(v.shape) if k == "layers.0.weight" else src)

    def state_dict(self) -> dict[str, torch.Tensor]:
        return {k: self._to_logical(k, v.detach()).clone().cpu() for k, v in self._logical(self.params).items()}

    def load_state_dict(self, sd: dict) -> None:
        self.params.zero_()
        self._load_logical(self.params, sd)
        if self.shadow is not None:
            self.shadow.copy_(self.params)

    def optimizer_state(self) -> dict:
        return {"m": {k: self._to_logical(k, v).clone().cpu() for k, v in self._logical(self.m).items()},
                "v": {k: self._to_logical(k, v).clone().cpu() for k, v in self._logical(self.v).items()},
                "step": int(self.state[0].item()), "hp": self.hp.cpu().tolist()}

    def load_optimizer_state(self, st: dict) -> None:
        self.m.zero_()
        self.v.zero_()
        for name, buf in (("m", self.m), ("v", self.v)):
            self._load_logical(buf, st[name])
        self.state[0] = int(st.get("step", 0))
        self.state[1] = 0

    def broadcast_parameters(self, src: int = 0, group=None) -> None:
        group = group if group is not None else self.group
        if group is None:
            return
        import torch.distributed as dist

        dist.broadcast(self.params, src=src, group=group)
        if self.shadow is not None:
            self.shadow.copy_(self.params)

    def average_parameters(self, group) -> None:
        """Spark ``ParameterAveragingTrainingMaster`` parity (``--avg-frequency``): the mean of the
        flat parameters and Adam moments over ``group`` (three flat all-reduces, no per-tensor calls)."""
        import torch.distributed as dist

        w = dist.get_world_size(group)
        for buf in (self.params, self.m, self.v):
            dist.all_reduce(buf, group=group)
            buf.mul_(1.0 / w)
        if self.shadow is not None:
            self.shadow.copy_(self.params)
