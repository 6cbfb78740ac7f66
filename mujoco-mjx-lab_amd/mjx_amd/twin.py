"""The PPO update's two networks as one batched pass per layer (train_ppo.py:233-252).

Per minibatch the reference takes a policy step (value_and_grad of ppo_loss_fn through the policy MLP)
and a value step (value_loss_fn through the value MLP), src/networks.py:22-131. With the reference's
src/config.json both MLPs have the same hidden layers (3 x 256 tanh) and read the same normalised
observations, so every hidden layer of the two nets is one strided-batched GEMM of batch 2 — twice the
tiles of one net's GEMM per launch — and every elementwise / reduction pass runs over both nets at
once. At the 8,192-row per-rank minibatch of C5 (8 GPUs) one net's 256-wide layer is 64 row tiles
for 256 CUs; the pair is 128, and the number of launches per minibatch step halves.

Layout (`TwinNets`): each layer's weights live in one stacked tensor W[l] [2, N, K] and b[l] [2, N]
(net 0 = policy, net 1 = value); the nn.Linear parameters of both modules become views of it, so
the rollout's packed policy, evaluation, checkpoints and the optimisers see the same storage. The
value's output layer (1 unit) is padded to the policy's A units with zero rows that receive zero
gradient (Adam leaves them at zero). The gradients land in one flat buffer laid out the same way,
which is also the data-parallel all-reduce buffer (no concatenation).

Forward: H_l = tanh(H_{l-1} W_lᵀ + b_l) as a bias-less torch.bmm + one native bias-and-tanh pass
(mjl_bias_act; baddbmm would first copy the broadcast bias into its output); Z = H W_outᵀ + b_out;
mean = tanh(Z[0]); v = Z[1][:, 0]. Losses and the output layers' dZ in one launch (mjl_twin_loss_head:
the clipped surrogate with log_std clipped in the kernel, the value's gradient 2 (v - ret) / M).
Backward, by hand in the order autograd takes: each layer's weight gradient is the split-K batched
GEMM dZᵀ X over both nets (2 x splits slices), its bias gradient the fixed-order column sums' first
stage (mjl_tanh_bwd_colsum_partials, which also forms dZ_l = dH (1 - H²)), dH = dZ W as one batched
GEMM; the second stages — every layer's slices and partials, the loss and d loss / d log_std
partials, summed in order — run together in one launch at the end (mjl_slice_sum_multi, which also
advances the captured update's counters). Same formulas as the per-net path (ppo.py _SplitKLinear /
_TanhSplitKLinear + the native losses); the GEMMs are the library's batched kernels instead of its
single ones, so results agree to rounding, not bit for bit (tests/test_twin.py)."""
from __future__ import annotations

import os
import weakref
from typing import List, Optional

import torch

from ._lib import check, lib

TWIN_UPDATE = os.environ.get("MJL_TWIN_UPDATE", "1") != "0"
# the output layers' bias + tanh inside the loss launch (mjl_twin_loss_head's bias argument) instead
# of a separate mjl_bias_act pass
FOLD_HEAD = os.environ.get("MJL_TWIN_FOLD_HEAD", "1") != "0"
# split-K slices of the 256-wide layers' weight gradients (None: the caller's splits), and of the thin
# ones (the 21-wide output, the 54-wide input; None: M / 256, at most 64)
HIDDEN_SPLITS = None
THIN_SPLITS = None
# rows per column-sum partial (the bias gradients' first stage); 32 and 64 measured no faster
COLSUM_CHUNK = int(os.environ.get("MJL_TWIN_COLSUM_CHUNK", "128"))
# the thin ends as single native launches where instantiated (csrc/twin_kernels.hip): the gather fused
# with both input layers (mjl_twin_gather_in), the output layers' backward fused with the last hidden
# layer's tanh backward (mjl_twin_head_bwd). MJL_TWIN_FUSED_ENDS=0: the library GEMM path for both
FUSED_ENDS = os.environ.get("MJL_TWIN_FUSED_ENDS", "1") != "0"
HEAD_BWD_ROWS = 128  # the fused output backward's row chunk (kHbRows)
HEAD_ROWS = 64  # the fused head takes row counts in multiples of this (its 32-row chunks, kThRows, divide it)
# MJL_TWIN_SIDE=1: the weight-gradient GEMMs on a second stream (fork / join inside the captured step),
# each layer's split-K dW = dZ^T X beside the main stream's dH = dZ W and the next tanh backward.
# Measured slower and off by default: C5's per-rank update 27.8 -> 33.5 ms (the fork / join events
# inside the graph cost more than the overlap gains)
SIDE_STREAM = os.environ.get("MJL_TWIN_SIDE", "0") == "1"
_SIDE = {}


def _side(dev):
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(dev)
    return s


# launch caps of the twin step's fused launches (csrc/ppo_loss_kernels.hip): mjl_adam_multi takes at most
# ADAM_MULTI_MAX_T tensors (the pair has 4 nl + 1: log_std plus a weight and a bias per layer of each
# net), mjl_slice_sum_multi at most SLICE_SEG_MAX segments (the pair has 2 nl + 2); deeper nets take
# the per-net path (tests/test_twin.py checks these against the kernel source)
ADAM_MULTI_MAX_T = 24
SLICE_SEG_MAX = 16


def _align4(n: int) -> int:
    return (n + 3) // 4 * 4


class TwinNets:
    """Stacked storage for a GaussianPolicy and a ValueNet with identical tanh hidden layers; builds
    the views and runs one minibatch's forward + backward into the flat gradient buffer."""

    @staticmethod
    def eligible(policy, value) -> bool:
        pm, vm = policy.mlp, value.mlp
        nl = len(pm.layers)
        if len(vm.layers) != nl or nl < 2 or 4 * nl + 1 > ADAM_MULTI_MAX_T or 2 * nl + 2 > SLICE_SEG_MAX:
            return False
        if not all(a == "tanh" for a in pm.acts[:-1]) or not all(a == "tanh" for a in vm.acts[:-1]):
            return False
        if pm.acts[-1] not in ("linear", "none") or vm.acts[-1] not in ("linear", "none"):
            return False
        for lp, lv in zip(pm.layers[:-1], vm.layers[:-1]):
            if lp.weight.shape != lv.weight.shape or lp.out_features % 4:
                return False
        A = pm.layers[-1].out_features
        ps = list(policy.parameters()) + list(value.parameters())
        # (A <= 31: the loss-head launch at 64 rows per block needs 2 A + 2 <= 64)
        return (vm.layers[-1].out_features == 1 and 1 <= A <= 31 and pm.layers[-1].in_features == vm.layers[-1].in_features
                and all(p.is_cuda and p.dtype == torch.float32 for p in ps) and policy.log_std.numel() == A)

    def __init__(self, policy, value):
        self.policy, self.value = policy, value
        pm, vm = policy.mlp, value.mlp
        dev = pm.layers[0].weight.device
        self.nl = len(pm.layers)
        self.A = pm.layers[-1].out_features
        self.K0 = pm.layers[0].in_features
        shapes = [tuple(l.weight.shape) for l in pm.layers]  # [N, K]; the output layer's N = A
        # one flat buffer for the stacked parameters and one for their gradients (+ log_std's)
        offs, o = [], 0
        for N, K in shapes:
            offs.append((o, _align4(o + 2 * N * K)))
            o = _align4(o + 2 * N * K) + _align4(2 * N)
        self.numel = o
        self.glog_off = o
        self.grad = torch.zeros(o + _align4(self.A), device=dev)
        self.store = torch.zeros(o, device=dev)
        self.W, self.b, self.gW, self.gb = [], [], [], []
        for (N, K), (ow, ob) in zip(shapes, offs):
            self.W.append(self.store[ow:ow + 2 * N * K].view(2, N, K))
            self.b.append(self.store[ob:ob + 2 * N].view(2, N))
            self.gW.append(self.grad[ow:ow + 2 * N * K].view(2, N, K))
            self.gb.append(self.grad[ob:ob + 2 * N].view(2, N))
        self.g_log_std = self.grad[self.glog_off:self.glog_off + self.A]
        with torch.no_grad():
            for l, (lp, lv) in enumerate(zip(pm.layers, vm.layers)):
                n_v = lv.out_features
                self.W[l][0].copy_(lp.weight)
                self.b[l][0].copy_(lp.bias)
                self.W[l][1, :n_v].copy_(lv.weight)
                self.b[l][1, :n_v].copy_(lv.bias)
                lp.weight.data = self.W[l][0]
                lp.bias.data = self.b[l][0]
                lv.weight.data = self.W[l][1, :n_v]
                lv.bias.data = self.b[l][1, :n_v]
        # gradient views in each module's parameters() order (the optimisers' order: a module's own
        # parameters come before its submodules', so GaussianPolicy yields log_std first)
        gview = {id(policy.log_std): self.g_log_std}
        for l in range(self.nl):
            n_v = vm.layers[l].out_features
            gview[id(pm.layers[l].weight)], gview[id(pm.layers[l].bias)] = self.gW[l][0], self.gb[l][0]
            gview[id(vm.layers[l].weight)], gview[id(vm.layers[l].bias)] = self.gW[l][1, :n_v], self.gb[l][1, :n_v]
        self.grads_p: List[torch.Tensor] = [gview[id(p)] for p in policy.parameters()]
        self.grads_v: List[torch.Tensor] = [gview[id(p)] for p in value.parameters()]
        self._scr = {}
        self.N0 = shapes[0][0]            # the first hidden width
        self.NH = shapes[-1][1]           # the last hidden width (the output layers' input)
        self._fused = int(lib().mjl_twin_fused_shapes(self.K0, self.A, self.N0)) & 1
        self._fused |= int(lib().mjl_twin_fused_shapes(self.K0, self.A, self.NH)) & 6

    def fused_input_ok(self, src) -> bool:
        """The gather + input layer launch applies: instantiated shape, the rollout arrays as the
        update passes them (f32, contiguous, the policy's widths)."""
        obs, acts = src[0], src[1]
        return (FUSED_ENDS and bool(self._fused & 1) and all(x.is_cuda and x.dtype == torch.float32 and x.is_contiguous()
                                                            for x in src)
                and obs.dim() == 2 and obs.shape[1] == self.K0 and acts.dim() == 2 and acts.shape[1] == self.A)

    def gather_input(self, idx, src, row: Optional[torch.Tensor] = None):
        """make_index_batches' rows of the rollout arrays (train_ppo.py:222-231) and both nets' first
        hidden layer in ONE launch (mjl_twin_gather_in): (o2 [2, M, K0] — the observations once per
        net —, acts [M, A], old_logp, ret, adv [M], h1 [2, M, N0] = tanh(o W0^T + b0)). With `row`
        (device int32) idx is the update's [n_minibatches, M] table, read at row *row when the launch
        runs (a captured minibatch step)."""
        obs, acts, logp, ret, adv = src
        idx = idx.contiguous()
        M = idx.shape[-1]
        dev = obs.device
        o2 = torch.empty((2, M, self.K0), device=dev)
        a = torch.empty((M, self.A), device=dev)
        ol, r, ad = (torch.empty(M, device=dev) for _ in range(3))
        h1 = torch.empty((2, M, self.N0), device=dev)
        nsrc = min(int(x.shape[0]) for x in src)
        check(lib().mjl_twin_gather_in(idx.data_ptr(), None if row is None else row.data_ptr(), M, nsrc, self.K0,
                                       self.A, self.N0, obs.data_ptr(), acts.data_ptr(), logp.data_ptr(),
                                       ret.data_ptr(), adv.data_ptr(), o2.data_ptr(), a.data_ptr(), ol.data_ptr(),
                                       r.data_ptr(), ad.data_ptr(), self.W[0].data_ptr(), self.b[0].data_ptr(),
                                       h1.data_ptr(), torch.cuda.current_stream(dev).cuda_stream))
        return o2, a, ol, r, ad, h1

    def owns_storage(self) -> bool:
        """Whether every parameter of both modules still is its view of the stacked storage (a
        load_state_dict copies into them and keeps it; re-assigning .data, load_state_dict(assign=True)
        or another TwinNets over the same modules would not): the update's forward reads the stacked
        tensors and Adam writes the modules' parameters, so both must be the same memory."""
        pm, vm = self.policy.mlp, self.value.mlp
        for l, (lp, lv) in enumerate(zip(pm.layers, vm.layers)):
            n_v = lv.out_features
            if (lp.weight.data_ptr() != self.W[l][0].data_ptr() or lp.bias.data_ptr() != self.b[l][0].data_ptr()
                    or lv.weight.data_ptr() != self.W[l][1, :n_v].data_ptr()
                    or lv.bias.data_ptr() != self.b[l][1, :n_v].data_ptr()):
                return False
        return True

    def _scratch(self, key, floats: int) -> torch.Tensor:
        st = torch.cuda.current_stream(self.grad.device).cuda_stream
        k = (key, floats, st)
        t = self._scr.get(k)
        if t is None:
            t = self._scr[k] = torch.empty(max(floats, 4), device=self.grad.device)
        return t

    def buckets(self):
        """The data-parallel all-reduce buffer in two buckets, in the order the backward completes them:
        bucket 1 = the top two layers of both nets and log_std (grad[o:], finished mid-backward), bucket
        2 = the layers below (grad[:o])."""
        o = self.gW[self.nl - 2].data_ptr() - self.grad.data_ptr()
        o //= self.grad.element_size()
        return self.grad[o:], self.grad[:o]

    def forward_backward(self, o, acts, old_logp, ret, adv, adv_stats, clip_eps: float, ent_coef: float, splits: int,
                         want_value_loss: bool = False, stats_row=None, counters=None, h1=None):
        """Both nets' losses and gradients for one minibatch (o [M, K0] — or [2, M, K0], the same rows
        twice, as the update's gather writes them —, acts [M, A], old_logp / ret / adv [M]); the
        gradients into self.grad. Returns (policy loss, value loss) device scalars (the value loss only
        with want_value_loss: the update does not need it). stats_row: adv_stats is the
        [n_minibatches, 2] table, read at that device row. counters: (policy step, value step, row)
        device counters that the final reduction launch advances (the captured update; Adam then runs
        with advanced=True)."""
        for out in self.forward_backward_phases(o, acts, old_logp, ret, adv, adv_stats, clip_eps, ent_coef, splits,
                                                want_value_loss, stats_row, counters, split=False, h1=h1):
            pass
        return out

    def forward_backward_phases(self, o, acts, old_logp, ret, adv, adv_stats, clip_eps: float, ent_coef: float,
                                splits: int, want_value_loss: bool = False, stats_row=None, counters=None,
                                split: bool = True, h1=None):
        """forward_backward as a generator. split: it yields None once bucket 1 of buckets() is final
        (the top two layers' weight-gradient slices and column-sum partials, the loss head's partials,
        summed in one launch), so the caller can start that bucket's all-reduce while the lower layers'
        backward runs (the data-parallel update's overlap); its last item is (policy loss, value
        loss) once bucket 2 -- and, with counters, the captured update's counters -- are final.
        h1: the first hidden layer's outputs from gather_input (o then is its [2, M, K0] copy)."""
        L = lib()
        dev = o.device
        st = torch.cuda.current_stream(dev).cuda_stream
        M, A, nl = o.shape[-2], self.A, self.nl
        s = splits
        # ---- forward: bias-less batched GEMMs, the bias and tanh in one native pass (mjl_bias_act).
        # Both nets read the same observations: a batch-stride-0 view, or the gathered copy per net
        # (which the first layer's weight-gradient slices can then read without an expand copy)
        x = o if o.dim() == 3 else o.unsqueeze(0).expand(2, M, self.K0)
        hs = [x] if h1 is None else [x, h1]
        # (the output layer's bias and tanh go into the loss launch unless the value loss is wanted)
        fold = FOLD_HEAD and not want_value_loss
        # the whole head as one launch (mjl_twin_head): the last hidden layer's bias + tanh, both output
        # layers, the losses and the head's backward down to that hidden layer's dZ
        whole_head = (FUSED_ENDS and fold and bool(self._fused & 4) and nl >= 2 and M % HEAD_ROWS == 0
                      and len(hs) <= nl - 1)
        zh = None
        for l in range(len(hs) - 1, nl):
            h = torch.bmm(hs[-1], self.W[l].transpose(1, 2))
            if whole_head and l == nl - 2:  # its bias and tanh inside the head launch; H never stored
                zh = h
                break
            mask = 3 if l < nl - 1 else 1  # the output layer: tanh for the policy's mean, linear value
            if l < nl - 1 or not fold:
                check(L.mjl_bias_act(h.data_ptr(), self.b[l].data_ptr(), 2, M, h.shape[2], mask, st))
            hs.append(h)
        z = None if whole_head else hs.pop()  # [2, M, A]: the policy's mean and the value in column 0 of
        # z[1] (fold: before the output bias and the mean's tanh)
        # ---- losses and the output layers' dZ in one launch (networks.py:103 clips log_std to [-20, 2]:
        # in the kernel, with its gradient mask); the value loss itself only for reporting.
        # Every reduction's first stage comes here (block partials of the loss, d loss / d log_std and
        # the output biases' gradients; the column-sum chunk partials and split-K weight-gradient slices
        # below); their second stages all in ONE launch after the last layer (mjl_slice_sum_multi)
        log_std = self.policy.log_std
        loss_p = torch.empty((), device=dev)
        loss_v = torch.empty((), device=dev)
        if want_value_loss:
            gv = torch.empty(M, device=dev)
            scr_v = self._scratch("mse", M // 256 + 1)
            check(L.mjl_mse_strided(z[1].data_ptr(), A, ret.data_ptr(), M, scr_v.data_ptr(), loss_v.data_ptr(),
                                    gv.data_ptr(), st))
        segs = []  # (x, out, nb, ns, m)
        scr = self._scratch("loss", int(L.mjl_ppo_loss_scratch(M, A)))
        if whole_head:
            K = self.W[nl - 1].shape[2]
            S = int(L.mjl_twin_head_blocks(M))
            dzh = torch.empty((2, M, K), device=dev)
            lossp, glsp = self._scratch("h_loss", S), self._scratch("h_gls", S * A)
            biasp, csp = self._scratch("h_bias", 2 * S * A), self._scratch("h_cs", 2 * S * K)
            gwp = self._scratch("h_gw", 2 * S * A * K)
            check(L.mjl_twin_head(zh.data_ptr(), self.b[nl - 2].data_ptr(), self.W[nl - 1].data_ptr(),
                                  self.b[nl - 1].data_ptr(), log_std.data_ptr(), acts.data_ptr(), old_logp.data_ptr(),
                                  adv.data_ptr(), ret.data_ptr(), None if adv_stats is None else adv_stats.data_ptr(),
                                  None if stats_row is None else stats_row.data_ptr(), M, A, K, float(clip_eps),
                                  float(ent_coef), -20.0, 2.0, scr.data_ptr(), dzh.data_ptr(), csp.data_ptr(),
                                  gwp.data_ptr(), lossp.data_ptr(), glsp.data_ptr(), biasp.data_ptr(), st))
            segs += [(lossp, loss_p, 1, S, 1), (glsp, self.g_log_std, 1, S, A), (biasp, self.gb[nl - 1], 2, S, A),
                     (gwp, self.gW[nl - 1], 2, S, A * K), (csp, self.gb[nl - 2], 2, S, K)]
            self._keep_head = (zh, dzh)
        else:
            dz = torch.empty((2, M, A), device=dev)
            nbk = int(L.mjl_twin_loss_head_blocks(M))
            part = self._scratch("lossparts", nbk * (1 + 3 * A))
            lossp, glsp, biasp = part[:nbk], part[nbk:nbk * (1 + A)], part[nbk * (1 + A):nbk * (1 + 3 * A)]
            check(L.mjl_twin_loss_head(z.data_ptr(), log_std.data_ptr(), acts.data_ptr(), old_logp.data_ptr(),
                                       adv.data_ptr(), ret.data_ptr(),
                                       None if adv_stats is None else adv_stats.data_ptr(),
                                       None if stats_row is None else stats_row.data_ptr(), M, A, float(clip_eps),
                                       float(ent_coef), -20.0, 2.0, self.b[nl - 1].data_ptr() if fold else None,
                                       scr.data_ptr(), dz.data_ptr(), lossp.data_ptr(),
                                       glsp.data_ptr(), biasp.data_ptr(), st))
            segs += [(lossp, loss_p, 1, nbk, 1), (glsp, self.g_log_std, 1, nbk, A),
                     (biasp, self.gb[nl - 1], 2, nbk, A)]
        # (32-row chunks — 4x the blocks — where the minibatch is small: 8.4 against 9.0 us per pass
        # at 8,192 rows; at 65,536 the 4x partials cost more than they gain)
        ch = COLSUM_CHUNK if M > 16384 else 32
        ch = ch if M % ch == 0 else M
        R = M // ch  # column-sum partial rows per matrix
        g = dzh if whole_head else dz
        main = torch.cuda.current_stream(dev)
        side = _side(dev) if SIDE_STREAM else None
        keep = []  # main-stream tensors the side stream reads: alive until the next step
        # the output layers' backward and the last hidden layer's tanh backward as one launch
        head_fused = FUSED_ENDS and bool(self._fused & 2) and nl >= 2 and M % HEAD_BWD_ROWS == 0
        for l in range(nl - 2 if whole_head else nl - 1, -1, -1):
            N, K = self.W[l].shape[1], self.W[l].shape[2]
            xin = hs[l]  # the layer's input: H_{l-1}, or the observations for l = 0
            if head_fused and l == nl - 1:  # dZ_{l-1}, its column-sum partials, this layer's dW partials
                R2 = M // HEAD_BWD_ROWS
                dzh = torch.empty((2, M, K), device=dev)
                csh = self._scratch("hb_cs", 2 * R2 * K)
                gwh = self._scratch("hb_gw", 2 * R2 * N * K)
                check(L.mjl_twin_head_bwd(g.data_ptr(), self.W[l].data_ptr(), xin.data_ptr(), M, N, K, dzh.data_ptr(),
                                          csh.data_ptr(), gwh.data_ptr(), st))
                segs.append((gwh, self.gW[l], 2, R2, N * K))
                segs.append((csh, self.gb[l - 1], 2, R2, K))
                g = dzh
                continue
            # split-K slices of the weight gradient: the thin layers (the 21 / 1-unit outputs, the 54-wide
            # input) are a few output tiles per slice, so they take more, shorter slices
            s = (HIDDEN_SPLITS or splits) if (N >= 64 and K >= 64) else max(splits, THIN_SPLITS or min(64, M // 256))
            if (head_fused or whole_head) and l == nl - 2:  # (its dZ and bias partials came from a fused launch)
                dzl = g
            elif l < nl - 1:  # tanh layer: dZ = dH (1 - H^2) and the bias gradient's partials in one pass
                dzl = torch.empty_like(g)
                cs = self._scratch(f"cs{l}", 2 * R * N)
                check(L.mjl_tanh_bwd_colsum_partials(g.data_ptr(), hs[l + 1].data_ptr(), 2, M, N, ch, dzl.data_ptr(),
                                                     cs.data_ptr(), st))
                segs.append((cs, self.gb[l], 2, R, N))
            else:
                dzl = g
            if l == 0 and o.dim() == 2:  # batch stride 0 -> per split, both nets (an expand copy)
                xs = o.view(1, s, M // s, K).expand(2, s, M // s, K).reshape(2 * s, M // s, K)
            else:
                xs = xin.view(2 * s, M // s, K)
            if side is not None:  # dW beside the main stream's dH and the next tanh backward
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    part = torch.bmm(dzl.view(2 * s, M // s, N).transpose(1, 2), xs)  # [2s, N, K]
                keep.append((dzl, xs))
            else:
                part = torch.bmm(dzl.view(2 * s, M // s, N).transpose(1, 2), xs)  # [2s, N, K]
            segs.append((part, self.gW[l], 2, s, N * K))
            if l > 0:
                g = torch.bmm(dzl, self.W[l])  # [2, M, K]
            if split and l == nl - 2:  # bucket 1 complete: its second stages now, then the caller's turn
                if side is not None:
                    main.wait_stream(side)
                self._slice_sum(segs, None, st)
                self._keep1 = (segs, hs, g)  # read by the launches in flight (and, captured, by the replays)
                segs = []
                yield None
        if side is not None:
            main.wait_stream(side)
        self._slice_sum(segs, counters, st)
        self._keep_side = keep
        yield loss_p, loss_v

    def _slice_sum(self, segs, counters, st):
        import ctypes
        k = len(segs)
        c0, c1, c2 = (None, None, None) if counters is None else (c.data_ptr() for c in counters)
        check(lib().mjl_slice_sum_multi(k, (ctypes.c_void_p * k)(*[x.data_ptr() for x, *_ in segs]),
                                        (ctypes.c_void_p * k)(*[o.data_ptr() for _, o, *_ in segs]),
                                        (ctypes.c_int * k)(*[nb for _, _, nb, _, _ in segs]),
                                        (ctypes.c_int * k)(*[ns for _, _, _, ns, _ in segs]),
                                        (ctypes.c_longlong * k)(*[m for *_, m in segs]), c0, c1, c2, st))
        self._keep = segs  # the launch reads the partial buffers asynchronously


def twin_for(policy, value) -> Optional[TwinNets]:
    """A TwinNets over (policy, value) when MJL_TWIN_UPDATE is on and the pair is eligible. The pair's
    TwinNets is cached per policy module (a weak-keyed table: no attribute on the module, nothing
    pulled along when it is pickled or copied) and reused while it still owns both modules' storage: a
    second TwinNets over the same modules would re-point their parameters and leave the first one's
    holder (a trainer's updater) on stale storage. Every updater built over the same pair therefore
    SHARES one TwinNets, including its scratch and kept-alive buffers: such updaters must not run
    concurrently (on different streams or threads)."""
    if not (TWIN_UPDATE and TwinNets.eligible(policy, value)):
        return None
    tw = _TWINS.get(policy)
    if tw is not None and tw.value is value and tw.owns_storage():
        return tw
    tw = TwinNets(policy, value)
    _TWINS[policy] = tw
    return tw


_TWINS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()  # policy module -> its TwinNets
