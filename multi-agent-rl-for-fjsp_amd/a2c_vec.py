"""Batched multi-agent A2C over N device-resident environments.

Reference: MultiAgentA2C (a2c.py:15-731) with networks.py.  Same networks (one actor per agent,
a centralised critic on the 38-dim global state), same predict rules (mask, renormalise,
uniform fallback, a2c.py:197-229), same memory / GAE (transition_memory.py:83-105), same
update (entropy bonus, per-agent advantage normalisation, gradient clipping, Adam,
a2c.py:647-731) and the same checkpoint format (a2c.py:733-775) — restated for N envs:

  * observations never leave HBM: the step kernel writes the a2c features f32 [38, N] and the
    post-reset masks int8 [29, N] of the next observation (fjsp_out.feats / next_masks), the
    policy reads them in place;
  * the 8 actors are one stacked module (weights [8, ...], inputs padded to 13 features and
    outputs to 8 actions): every layer is ONE batched GEMM (torch.baddbmm -> hipBLASLt) for
    all agents and envs instead of 8 x N GEMVs;
  * one update per `batch_size` vector steps uses all batch_size x N transitions; the loss
    means / advantage statistics are over that whole batch (for N = 1 this is exactly the
    reference's update);
  * multi-GPU (config 5): every rank steps its own env shard (envs keyed by global id: MT
    streams and action draws), then either computes local sums and one bucketed all_reduce
    (RCCL) of the gradients (exchange="allreduce", default) or gathers its transitions into the
    learner rank, which updates over the whole batch and broadcasts the parameters
    (exchange="gather", the reference's memory -> finish_trajectory -> _update); both equal a
    single learner over all ranks' transitions (distributed.py).

Padding is exact: padded input columns are zero and their weights receive zero gradient;
padded action logits are -inf before the softmax.
"""
import ctypes
import os
import math

import torch
from torch import nn

from . import _native as nat
from .spec import AGENTS, N_ACTIONS

NA = 8
OBS_DIMS = [7, 13, 3, 3, 3, 3, 3, 3]          # _get_obs_dim per agent (a2c.py:118-134)
OBS_OFFS = [0, 7, 20, 23, 26, 29, 32, 35]      # agent blocks of the 38-dim global state
MASK_OFFS = [0, 3, 11, 14, 17, 20, 23, 26]     # agent blocks of the 29 mask bytes
MASK_DIM = 29
GLOBAL_DIM = 38
DPAD, APAD = 13, 8


# ---------------------------------------------------------------- reference-shaped networks
class ActorNet(nn.Module):
    """networks.ActorNetwork layout (state_dict keys net.0/2/4.*)."""

    def __init__(self, d, a, hidden=256):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(d, hidden), nn.ReLU(), nn.Linear(hidden, hidden), nn.ReLU(),
                                 nn.Linear(hidden, a), nn.Softmax(dim=-1))

    def forward(self, x):
        return self.net(x)


class CriticNet(nn.Module):
    """networks.CentralizedCriticNetwork layout (state_dict keys net.0/2/4/6.*)."""

    def __init__(self, d, hidden=256):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(d, hidden), nn.ReLU(), nn.Linear(hidden, hidden), nn.ReLU(),
                                 nn.Linear(hidden, hidden // 2), nn.ReLU(), nn.Linear(hidden // 2, 1))

    def forward(self, x):
        return self.net(x)


class _LinearSplitK(torch.autograd.Function):
    """y = x W^T + b (relu: max(y, 0) in the GEMM's epilogue) whose weight gradient over a long
    batch is a batched GEMM over batch chunks summed afterwards (split-K): one [out, in] GEMM
    with K = 10^5..10^6 samples leaves most of the chip idle (a few dozen output tiles).  The
    input gradient is skipped when x needs none (the first layer)."""

    @staticmethod
    def forward(ctx, x, W, b, relu):
        y = torch._addmm_activation(b, x, W.t()) if relu else torch.addmm(b, x, W.t())
        ctx.relu = relu
        ctx.save_for_backward(x, W, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, W, y = ctx.saved_tensors
        gb = None
        if ctx.relu and gy.is_cuda and W.shape[0] in (128, 256):
            gy, gb = _relu_bias_grad(gy.contiguous(), y)            # one pass (HIP kernel)
        elif ctx.relu:
            gy = torch.ops.aten.threshold_backward(gy, y, 0.0)      # relu' from the output
        gW = critic_wgrad(gy, x) if _wgrad_fits(gy, x) else _splitk_wgrad(gy, x)
        gx = None
        if ctx.needs_input_grad[0]:
            # one output (the value head): an outer product, elementwise (a K = 1 GEMM is slow)
            gx = gy * W if W.shape[0] == 1 else gy @ W
        return gx, gW, gy.sum(0) if gb is None else gb, None


def _critic_wgrad(gy, x, nx=None):
    """A critic layer's weight gradient gy^T x[:, :nx]: on the GPU one fjsp_a2c_wgrad launch (the
    samples' contraction on the matrix cores, f32-level products, deterministic; r06), else the
    split-K GEMM."""
    if gy.is_cuda and wgrad_kernel_on:
        return critic_wgrad(gy, x, nx)
    return _splitk_wgrad(gy, x if nx is None else x[:, :nx])


wgrad_kernel_on = True   # False: the critic's weight gradients as split-K hipBLASLt GEMMs (A/B)


def _wgrad_fits(gy, x):
    """fjsp_a2c_wgrad takes this gy^T x (contiguous rows, a supported layer shape): the critic's
    layers and the long-batch actor's 256-wide hidden layer (_LinearSplitK)."""
    if not (gy.is_cuda and wgrad_kernel_on and gy.dim() == 2 and x.dim() == 2 and gy.is_contiguous()
            and x.is_contiguous() and x.shape[1] % 4 == 0):
        return False
    m, nx = gy.shape[1], x.shape[1]
    return (m in (128, 256) and 68 <= nx <= 256) or (m == 256 and 4 <= nx <= 64)


def critic_wgrad(g, x, nout=None, parts=None):
    """fjsp_a2c_wgrad: g f32 [U, m] (m = 256 / 128), x f32 [U, nx] rows (both contiguous, nx % 4 == 0)
    -> g^T x[:, :nout] f32 [m, nout]."""
    U, m = g.shape
    nx = x.shape[1]
    nout = nx if nout is None else nout
    g, x = g.contiguous(), x.contiguous()
    npad = 256 if nx > 64 else 64
    if parts is None:   # one workgroup per CU (the double-buffered images take 90-144 KB of LDS)
        parts = 256
    # the kernel's buffer offsets are 32-bit: longer batches in chunks, summed in order
    rows = min(WGRAD_MAX_ROWS, (0x7FFFFF00 // (4 * max(m, nx))) - 5 * parts * 16)
    part = torch.empty(parts, m, npad, dtype=torch.float32, device=g.device)
    V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream(g.device).cuda_stream)
    out = None
    for r0 in range(0, U, rows):
        n = min(rows, U - r0)
        o = torch.empty(m, nout, dtype=torch.float32, device=g.device)
        nat.check(nat.lib().fjsp_a2c_wgrad(V(g[r0:]), m, m, V(x[r0:]), nx, nx, n, V(part), parts, V(o), nout, nout, st))
        out = o if out is None else out.add_(o)
    return out


WGRAD_MAX_ROWS = 1 << 40   # chunk size cap (tests lower it to exercise the chunked path)


def _splitk_wgrad(gy, x):
    """gy^T x over a long batch B: c chunks of B // c rows as strided views (no padded copies)
    in one batched GEMM, summed; the B - c * (B // c) tail apart."""
    B = x.shape[0]
    c = max(1, min(128, B // 8192))   # 128 chunks: 7 % faster than 64 at U = 698 k (profiles/r06/a2c/ab_wgrad_split.json)
    bc = B // c
    xc = x[:c * bc].reshape(c, bc, -1)
    gc = gy[:c * bc].reshape(c, bc, -1)
    if x.stride(0) == 1:   # x a transposed [in, B] slab (the first layer): (x^T g)^T, both operands natural
        gW = torch.bmm(xc.transpose(1, 2), gc).sum(0).t()
    else:
        gW = torch.bmm(gc.transpose(1, 2), xc).sum(0)
    if c * bc < B:
        gW += gy[c * bc:].t() @ x[c * bc:]
    return gW


class _ValueHead(torch.autograd.Function):
    """The critic's last two layers v = relu(h W3^T + b3) w4^T + b4 over a long batch on the
    GPU; backward: layer 3's ReLU and bias gradient, the value head's weight and bias gradient
    and the gradient into layer 3 in one pass over the 128-wide activations
    (fjsp_a2c_value_head_grad), then layer 3's split-K weight gradient."""

    @staticmethod
    def forward(ctx, h, W3, b3, W4, b4):
        y = torch._addmm_activation(b3, h, W3.t())
        ctx.save_for_backward(h, W3, y, W4)
        return torch.addmm(b4, y, W4.t())

    @staticmethod
    def backward(ctx, gv):
        h, W3, y, W4 = ctx.saved_tensors
        B, C = y.shape
        gvc = gv.reshape(-1).contiguous()
        w4 = W4.reshape(-1).contiguous()
        g = torch.empty_like(y)
        part = torch.empty(-(-B // 128), 2 * C + 4, dtype=torch.float32, device=y.device)
        stream = torch.cuda.current_stream(y.device).cuda_stream
        V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        nat.check(nat.lib().fjsp_a2c_value_head_grad(V(y), V(gvc), V(w4), B, V(g), V(part), ctypes.c_void_p(stream)))
        ps = part.sum(0)
        gh = g @ W3 if ctx.needs_input_grad[0] else None
        return gh, _splitk_wgrad(g, h), ps[:C], ps[C:2 * C].view(1, C), ps[2 * C:2 * C + 1]


def _relu_bias_grad(gy, y):
    """(gy where y > 0 else 0, its column sums) for y [B, C] = a ReLU output, gy [B, C]
    contiguous f32 on the GPU: fjsp_a2c_relu_bias_grad."""
    B, C = y.shape
    g = torch.empty_like(gy)
    part = torch.empty(-(-B // 128), C, dtype=torch.float32, device=gy.device)
    stream = torch.cuda.current_stream(gy.device).cuda_stream
    V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    nat.check(nat.lib().fjsp_a2c_relu_bias_grad(V(gy), V(y), B, C, V(g), V(part), ctypes.c_void_p(stream)))
    return g, part.sum(0)


class _CriticGrouped(torch.autograd.Function):
    """The critic (38 -> 256 -> 256 -> 128 -> 1, ReLUs) over a long batch of distinct global states
    on the GPU: the forward in one fused kernel (fjsp_a2c_critic_forward: f32 operands as bf16
    planes on the matrix cores, as the policy kernel's values), which also writes the hidden
    layers; the backward: the value-head kernel, both 256-wide ReLU layers' input gradients in one
    kernel (fjsp_a2c_critic_backward, the same split arithmetic), split-K weight gradients
    (hipBLASLt; a matrix-core kernel for them measured slower).
    x f32 [U, 40] (sample-major rows: 38 features, 2 zeros) -> v [U]."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2, W3, b3, W4, b4):
        U = x.shape[0]
        dev = x.device
        cw = pack_critic_weights(W1, b1, W2, b2, W3, b3, W4, b4)
        h1 = torch.empty(U, W2.shape[1], dtype=torch.float32, device=dev)
        h2 = torch.empty(U, W2.shape[0], dtype=torch.float32, device=dev)
        h3 = torch.empty(U, W3.shape[0], dtype=torch.float32, device=dev)
        v = torch.empty(U, dtype=torch.float32, device=dev)
        V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        stream = torch.cuda.current_stream(dev).cuda_stream
        nat.check(nat.lib().fjsp_a2c_critic_forward(V(x), U, V(cw), V(h1), V(h2), V(h3), V(v), ctypes.c_void_p(stream)))
        ctx.save_for_backward(x, W2, W3, W4, h1, h2, h3)
        return v

    @staticmethod
    def backward(ctx, gv):
        x, W2, W3, W4, h1, h2, h3 = ctx.saved_tensors
        B, C = h3.shape
        gvc = gv.reshape(-1).contiguous()
        w4 = W4.reshape(-1).contiguous()
        g3 = torch.empty_like(h3)
        part = torch.empty(-(-B // 128), 2 * C + 4, dtype=torch.float32, device=h3.device)
        stream = torch.cuda.current_stream(h3.device).cuda_stream
        V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        nat.check(nat.lib().fjsp_a2c_value_head_grad(V(h3), V(gvc), V(w4), B, V(g3), V(part), ctypes.c_void_p(stream)))
        ps = part.sum(0)
        gW3 = _splitk_wgrad(g3, h2)
        if critic_bwd_fused:
            # both 256-wide ReLU layers' input gradients in one pass (fjsp_a2c_critic_backward)
            w3t, w2t = pack_mfma(W3.detach().t()).reshape(-1), pack_mfma(W2.detach().t()).reshape(-1)
            g2, g1 = torch.empty_like(h2), torch.empty_like(h1)
            nt = -(-B // 32)
            bp2 = torch.empty(nt, h2.shape[1], dtype=torch.float32, device=h2.device)
            bp1 = torch.empty(nt, h1.shape[1], dtype=torch.float32, device=h1.device)
            nat.check(nat.lib().fjsp_a2c_critic_backward(V(g3), V(h1), V(h2), B, V(w3t), V(w2t), V(g2), V(g1), V(bp2),
                                                         V(bp1), ctypes.c_void_p(stream)))
            gb2, gb1 = bp2.sum(0), bp1.sum(0)
        else:
            g2, gb2 = _relu_bias_grad((g3 @ W3).contiguous(), h2)
            g1, gb1 = _relu_bias_grad((g2 @ W2).contiguous(), h1)
        gW2 = _splitk_wgrad(g2, h1)
        gW1 = _splitk_wgrad(g1, x[:, :GLOBAL_DIM])
        return (None, gW1, gb1, gW2, gb2, gW3, ps[:C], ps[C:2 * C].view(1, C), ps[2 * C:2 * C + 1])


class _CriticOnePass(torch.autograd.Function):
    """The grouped update's critic loss and its gradients in one kernel pass over the distinct
    global states (fjsp_a2c_critic_fused: forward, value gradient from the per-state loss
    coefficients, value head and the two 256-wide layers' backward; a2c.py:683-699, 713-722); the
    three split-K weight gradients in backward (a loss-only call pays for none of them).  x f32
    [U, 40] (sample-major rows), coef f64 [U, 3] = (a, b, c) with state u's loss a/2 V^2 + b V + c
    (critic_coef) -> the critic loss (0-d f32); backward returns the gradients, scaled by the
    loss's gradient."""

    @staticmethod
    def forward(ctx, x, coef, W1, b1, W2, b2, W3, b3, W4, b4):
        loss, ctx.parts = critic_onepass_compute(x, coef, W1, b1, W2, b2, W3, b3, W4, b4)
        return loss

    @staticmethod
    def backward(ctx, gl):
        grads = critic_onepass_grads(*ctx.parts)
        ctx.parts = None
        return (None, None) + tuple(torch._foreach_mul(list(grads), gl))


@torch.no_grad()
def critic_onepass_grads(x, h1, h2, g1, g2, g3, ps):
    """The critic's gradients W1, b1, W2, b2, W3, b3, W4, b4 from fjsp_a2c_critic_fused's outputs."""
    return (_critic_wgrad(g1, x, GLOBAL_DIM), ps[:256], _critic_wgrad(g2, h1), ps[256:512],
            _critic_wgrad(g3, h2), ps[512:640], ps[640:768].view(1, 128), ps[768:769])


@torch.no_grad()
def critic_onepass_compute(x, coef, W1, b1, W2, b2, W3, b3, W4, b4):
    """_CriticOnePass's kernel pass on the current stream: (the critic loss 0-d f32, the inputs of
    critic_onepass_grads: x and the per-state activations / activation gradients the kernel wrote,
    and the per-tile bias / value-head partial sums summed)."""
    U = x.shape[0]
    dev = x.device
    cw = pack_critic_weights(W1, b1, W2, b2, W3, b3, W4, b4)
    w3t, w2t = pack_mfma(W3.detach().t()).reshape(-1), pack_mfma(W2.detach().t()).reshape(-1)
    E = lambda *sh: torch.empty(*sh, dtype=torch.float32, device=dev)  # noqa: E731
    h1, h2, g2, g1, g3 = E(U, 256), E(U, 256), E(U, 256), E(U, 256), E(U, 128)
    tiles = -(-U // 32)
    part = E(tiles, nat.CRITIC_FUSED_PW)
    loss = torch.empty(tiles, dtype=torch.float64, device=dev)
    V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    c = coef.contiguous()
    nat.check(nat.lib().fjsp_a2c_critic_fused(V(x), U, V(cw), V(w3t), V(w2t), V(c), V(h1), V(h2), V(g3), V(g2),
                                              V(g1), V(part), V(loss), None,
                                              ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    return loss.sum().float(), (x, h1, h2, g1, g2, g3, part.sum(0))


def slab_stats(ret=None, adv=None):
    """fjsp_a2c_slab_stats over the GAE outputs f64 [T, 8, N] (GPU): (rs f64 [2, T*N] = per sample the
    sums over the agents of the f32-rounded return and of its square, or None; sums f64 [8, 2] = per
    agent the sums of the f32-rounded advantage and of its square, or None)."""
    x = ret if ret is not None else adv
    T, _, N = x.shape
    dev = x.device
    V = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
    rs = torch.empty(2, T * N, dtype=torch.float64, device=dev) if ret is not None else None
    part = torch.empty(T, -(-N // 256), NA, 2, dtype=torch.float64, device=dev) if adv is not None else None
    r = None if ret is None else ret.contiguous()
    a = None if adv is None else adv.contiguous()
    nat.check(nat.lib().fjsp_a2c_slab_stats(V(r), V(a), T, N, None if rs is None else V(rs[0]),
                                            None if rs is None else V(rs[1]), V(part),
                                            ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    return rs, None if part is None else part.sum(dim=(0, 1))


def critic_coef(g, r3, count):
    """Per distinct global state u of the (device) RowGroups g (one row: the critic's grouping of
    the batch's S = T * n samples) the coefficients of its share of calc_critic_loss
    (a2c.py:713-722): sum over its n_u samples and the 8 agents of (V_u - R)^2 / (8 count) =
    a/2 V^2 + b V + c, a = 2 n_u / count, b = -2 sum R / (8 count), c = sum R^2 / (8 count), R the
    f32 returns (r3 f64 [T, 8, n]) summed in f64 in sorted order -> f64 [Umax, 3]."""
    from .shard_learner import _counts, _group_sums
    if r3.is_cuda:
        rs, _ = slab_stats(ret=r3)                                                        # [2, S]
    else:
        r32 = r3.float().double()
        S = r32.shape[0] * r32.shape[2]
        rs = torch.stack([r32.sum(1).reshape(S), (r32 * r32).sum(1).reshape(S)])
    sums = _group_sums(g.perm, g.ends, rs)                                                # [2, Umax]
    return critic_coef_sums(_counts(g.ends)[0].double(), sums[0], sums[1], count)


def critic_coef_sums(nu, sr, sr2, count):
    """critic_coef from per-state sample counts and sums of R and R^2 (f64 [U] each)."""
    return torch.stack([2.0 * nu / count, -2.0 * sr / (NA * count), sr2 / (NA * count)], dim=1).contiguous()


def critic_onepass(critic, x, coef):
    """The critic loss over distinct states x f32 [U, 40] with coefficients coef f64 [U, 3]
    (critic_coef), gradients through _CriticOnePass."""
    n = critic.net
    assert x.shape[1] == GROUP_ROW
    return _CriticOnePass.apply(x.contiguous(), coef, n[0].weight, n[0].bias, n[2].weight, n[2].bias, n[4].weight,
                                n[4].bias, n[6].weight, n[6].bias)


# Implementation switches of the grouped update (module attributes, set from Python by the A/B
# scripts and the tests; every setting computes the same losses and gradients):
# the critic through the fused forward kernel (False: PyTorch GEMMs)
critic_fused = True
# ... and its loss, forward and backward in one pass per distinct state (fjsp_a2c_critic_fused;
# False: the forward kernel, the per-sample loss through autograd, the value head and backward kernels)
critic_onepass_on = True

# its backward through the two 256-wide layers in one kernel (False: GEMMs + ReLU kernels)
critic_bwd_fused = True


def feature_rows(f3):
    """feats f32 [T, 38, N] -> the sample-major rows f32 [T*N, 40] (zero-padded) that
    group_keys writes on the GPU (for callers without them)."""
    T, _, N = f3.shape
    return torch.nn.functional.pad(f3.permute(0, 2, 1).reshape(T * N, GLOBAL_DIM),
                                   (0, GROUP_ROW - GLOBAL_DIM)).contiguous()


def critic_grouped(critic, x):
    """v [U] of the critic over the rows of x f32 [U, 40] (distinct global states, sample-major,
    38 features + 2 zeros: feature_rows / group_keys' rows)."""
    n = critic.net
    assert x.shape[1] == GROUP_ROW
    return _CriticGrouped.apply(x.contiguous(), n[0].weight, n[0].bias, n[2].weight, n[2].bias, n[4].weight,
                                n[4].bias, n[6].weight, n[6].bias)


def mlp_forward(seq, x):
    """An nn.Sequential of Linear / ReLU on x [B, in] with split-K weight gradients and the
    ReLU fused into the GEMM for long batches (the same parameters, the same math)."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        if (x.is_cuda and x.shape[0] >= 65536 and i + 3 == len(mods) and isinstance(m, nn.Linear)
                and isinstance(mods[i + 1], nn.ReLU) and isinstance(mods[i + 2], nn.Linear)
                and mods[i + 2].out_features == 1 and m.out_features == 128):
            return _ValueHead.apply(x, m.weight, m.bias, mods[i + 2].weight, mods[i + 2].bias)
        if isinstance(m, nn.Linear) and x.shape[0] >= 65536:
            relu = i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
            x = _LinearSplitK.apply(x, m.weight, m.bias, relu)
            i += 2 if relu else 1
        else:
            x = m(x)
            i += 1
    return x


class ActorStack(nn.Module):
    """The 8 ActorNetworks as stacked, padded weights; forward is 3 batched GEMMs.

    Layout "agent-major, batch last": x [8, 13, B] -> logits [8, 8, B]; the batch dimension is
    the GEMM's N dimension so the kernel-written [38, N] features feed it without a transpose.
    """

    def __init__(self, hidden=256):
        super().__init__()
        self.hidden = hidden
        self.W1 = nn.Parameter(torch.zeros(NA, hidden, DPAD))
        self.b1 = nn.Parameter(torch.zeros(NA, hidden, 1))
        self.W2 = nn.Parameter(torch.zeros(NA, hidden, hidden))
        self.b2 = nn.Parameter(torch.zeros(NA, hidden, 1))
        self.W3 = nn.Parameter(torch.zeros(NA, APAD, hidden))
        self.b3 = nn.Parameter(torch.zeros(NA, APAD, 1))
        pad = torch.full((NA, APAD, 1), float("-inf"))
        for a, n in enumerate(N_ACTIONS):
            pad[a, :n] = 0.0
        self.register_buffer("logit_pad", pad)

    def logits(self, x):
        h = torch.relu(torch.baddbmm(self.b1, self.W1, x))
        h = torch.relu(torch.baddbmm(self.b2, self.W2, h))
        return torch.baddbmm(self.b3, self.W3, h) + self.logit_pad

    def forward(self, x):
        return torch.softmax(self.logits(x), dim=1)

    def agent_probs(self, a, x):
        """Actor a alone on x [13, B] -> probabilities [8, B] (the agent's slice of forward);
        a long batch through the split-K layers (a weight gradient with K = B and a [256, 13]
        output is a handful of GEMM tiles)."""
        if x.shape[1] >= 16384:
            h = _LinearSplitK.apply(x.t(), self.W1[a], self.b1[a, :, 0], True)
            h = _LinearSplitK.apply(h, self.W2[a], self.b2[a, :, 0], True)
            z = _LinearSplitK.apply(h, self.W3[a], self.b3[a, :, 0], False)
            return torch.softmax(z.t() + self.logit_pad[a], dim=0)
        h = torch.relu(torch.addmm(self.b1[a], self.W1[a], x))
        h = torch.relu(torch.addmm(self.b2[a], self.W2[a], h))
        return torch.softmax(torch.addmm(self.b3[a], self.W3[a], h) + self.logit_pad[a], dim=0)

    def forward_rows(self, x, g, cols=None):
        """The actors on their agents' distinct inputs: x [8, 13, S], g = RowGroups of the
        agents' keys -> probabilities [8, 8, Umax] per group.  The agent with the most groups
        runs alone and the others stacked on the second-largest count (padding columns are
        computed and never gathered).  cols(agents, idx [k, u]) -> [k, 13, u] may stand in for x
        (the inputs of just the representatives)."""
        U = g.U
        umax = g.first.shape[1]
        big = max(range(NA), key=lambda a: U[a])
        rest = [a for a in range(NA) if a != big]
        u2 = bucket(max(U[a] for a in rest))
        ub = bucket(U[big])
        ridx = _index_tensor(tuple(rest), g.first.device)
        fr = g.first[ridx, :u2]
        if cols is None:
            xr = torch.gather(x[ridx], 2, fr[:, None, :].expand(NA - 1, x.shape[1], u2))
            xb = x[big][:, g.first[big, :ub]]
        else:
            xr = cols(ridx, fr)
            xb = cols(_index_tensor((big,), ridx.device), g.first[big:big + 1, :ub])[0]
        h = torch.relu(torch.baddbmm(self.b1[ridx], self.W1[ridx], xr))
        h = torch.relu(torch.baddbmm(self.b2[ridx], self.W2[ridx], h))
        pr = torch.softmax(torch.baddbmm(self.b3[ridx], self.W3[ridx], h) + self.logit_pad[ridx], dim=1)
        pb = self.agent_probs(big, xb)
        # rest is range(NA) without big, in order: the stacked agents around the big one (three
        # launches; eight pads and a stack before)
        pr = torch.nn.functional.pad(pr, (0, umax - u2))
        pb = torch.nn.functional.pad(pb, (0, umax - ub))[None]
        return torch.cat([pr[:big], pb, pr[big:]])

    def forward_grouped(self, x, keys=None):
        """forward on x [8, 13, S], each actor run once per distinct observation of its agent,
        the probabilities gathered back per sample (A2CLosses dedup); keys [8, S] = row_keys(x)."""
        g = RowGroups(row_keys(x) if keys is None else keys)
        if not bool((torch.gather(x, 2, g.rep[:, None, :].expand_as(x)) == x).all()):
            return self(x)
        return g.gather(self.forward_rows(x, g))

    @torch.no_grad()
    def load_actor_nets(self, nets):
        for a, net in enumerate(nets):
            l1, l2, l3 = net.net[0], net.net[2], net.net[4]
            d, n = OBS_DIMS[a], N_ACTIONS[a]
            self.W1[a].zero_(); self.W1[a, :, :d].copy_(l1.weight)
            self.b1[a, :, 0].copy_(l1.bias)
            self.W2[a].copy_(l2.weight); self.b2[a, :, 0].copy_(l2.bias)
            self.W3[a].zero_(); self.W3[a, :n].copy_(l3.weight)
            self.b3[a].zero_(); self.b3[a, :n, 0].copy_(l3.bias)

    @torch.no_grad()
    def actor_state_dict(self, a):
        d, n = OBS_DIMS[a], N_ACTIONS[a]
        c = lambda t: t.detach().cpu().clone()  # noqa: E731
        return {"net.0.weight": c(self.W1[a, :, :d]), "net.0.bias": c(self.b1[a, :, 0]),
                "net.2.weight": c(self.W2[a]), "net.2.bias": c(self.b2[a, :, 0]),
                "net.4.weight": c(self.W3[a, :n]), "net.4.bias": c(self.b3[a, :n, 0])}


def gather_index(device):
    """[8, 13] row indices into [features(38) | zero row] building the padded actor inputs."""
    idx = torch.full((NA, DPAD), GLOBAL_DIM, dtype=torch.long)
    for a in range(NA):
        idx[a, :OBS_DIMS[a]] = torch.arange(OBS_OFFS[a], OBS_OFFS[a] + OBS_DIMS[a])
    return idx.to(device)


def mask_index(device):
    """[8, 8] indices into [masks(29) | zero row] -> per-agent padded masks."""
    idx = torch.full((NA, APAD), 29, dtype=torch.long)
    for a in range(NA):
        idx[a, :N_ACTIONS[a]] = torch.arange(MASK_OFFS[a], MASK_OFFS[a] + N_ACTIONS[a])
    return idx.to(device)


# ---------------------------------------------------------------- policy math (any device)
def actor_inputs(feats, gidx):
    """feats f32 [..., 38, B] -> padded actor inputs [8, 13, (...)*B]."""
    lead = feats.shape[:-2]
    B = feats.shape[-1]
    z = torch.zeros(*lead, 1, B, dtype=feats.dtype, device=feats.device)
    x = torch.cat([feats, z], dim=-2)[..., gidx, :]                 # [..., 8, 13, B]
    if lead:
        x = x.reshape(-1, NA, DPAD, B).permute(1, 2, 0, 3).reshape(NA, DPAD, -1)
    return x


def agent_masks(masks, midx):
    """int8 masks [..., 29, B] -> float [8, 8, (...)*B] (padded actions are 0)."""
    lead = masks.shape[:-2]
    B = masks.shape[-1]
    z = torch.zeros(*lead, 1, B, dtype=torch.float32, device=masks.device)
    m = torch.cat([masks.to(torch.float32), z], dim=-2)[..., midx, :]
    if lead:
        m = m.reshape(-1, NA, APAD, B).permute(1, 2, 0, 3).reshape(NA, APAD, -1)
    return m


def masked_probs(probs, mask):
    """a2c.py:204-220: zero invalid actions, renormalise; if nothing is left, uniform over
    the valid actions."""
    p = probs * mask
    s = p.sum(dim=1, keepdim=True)
    uni = mask / mask.sum(dim=1, keepdim=True)
    return torch.where(s > 0, p / torch.where(s > 0, s, torch.ones_like(s)), uni)


def categorical_log_prob(p, actions):
    """Categorical(probs=p).log_prob(actions) batched, written out (no argument validation,
    which would synchronise): probs / sum -> log(clamp(eps, 1 - eps)) -> gather.
    p [8, 8, B], actions long [8, B] -> [8, B]."""
    q = p / p.sum(dim=1, keepdim=True)
    eps = torch.finfo(q.dtype).eps
    return torch.log(q.clamp(min=eps, max=1 - eps)).gather(1, actions.unsqueeze(1)).squeeze(1)


_M64 = (1 << 64) - 1


def _fmix64(z):
    """splitmix64's finaliser on int64 tensors (wrapping multiply, logical shifts): the same
    hash csrc/fjsp_policy.hip draws its actions with."""
    def shr(x, k):
        return (x >> k) & ((1 << (64 - k)) - 1)

    def s64(c):
        return c - (1 << 64) if c >= (1 << 63) else c
    z = z ^ shr(z, 30)
    z = z * s64(0xBF58476D1CE4E5B9)
    z = z ^ shr(z, 27)
    z = z * s64(0x94D049BB133111EB)
    return z ^ shr(z, 31)


def _s64(c):
    c &= _M64
    return c - (1 << 64) if c >= (1 << 63) else c


_ROLE_KEYS = {}


def role_keys(device):
    """The per-agent keys (a + 1) * golden-ratio of the policy draw, int64 [8] on `device`
    (built once per device: a host-to-device copy must not happen inside a graph capture)."""
    device = torch.device(device)
    if device not in _ROLE_KEYS:
        _ROLE_KEYS[device] = torch.tensor([_s64((a + 1) * 0x9E3779B97F4A7C15) for a in range(NA)],
                                          dtype=torch.int64, device=device)
    return _ROLE_KEYS[device]


def counter_uniform(seed, gid, step, device):
    """U [8, 1, B] in [0, 1) keyed by (seed, global env id, step, agent) exactly as the fused
    policy kernel's draw (fjsp_policy.hip): shards of a multi-GPU job draw independent streams
    and the eager and fused paths see the same uniforms.  seed: a Python int or an int64
    tensor of one element on `device` (read at run time: a captured graph re-keys with it)."""
    g = torch.as_tensor(gid, device=device).to(torch.int64) & 0xFFFFFFFF
    inner = _fmix64((g << 32) | (int(step) & 0xFFFFFFFF))
    s = seed.reshape(1) if torch.is_tensor(seed) else _s64(seed)
    h = _fmix64((s ^ inner)[None, :] ^ role_keys(device)[:, None])         # [8, B]
    return ((h >> 40) & 0xFFFFFF).to(torch.float32).mul_(1.0 / 16777216.0).unsqueeze(1)


def sample_categorical(p, u=None):
    """One draw per (agent, env) from p [8, 8, B] by inverse CDF: action = #{k : cdf_k < x}
    with x = (1 - U) * cdf_last, U ~ [0, 1) -> x in (0, total]; a zero-probability action can
    never be returned (its CDF step is empty), padded actions neither."""
    if u is None:
        u = torch.rand(p.shape[0], 1, p.shape[2], device=p.device, dtype=p.dtype)
    cdf = torch.cumsum(p, dim=1)
    x = (1.0 - u) * cdf[:, -1:, :]
    return (cdf < x).sum(dim=1)


def entropy_of(probs):
    """_calculate_entropy (a2c.py:705-722): -(p * log(p + 1e-10)).sum() per observation."""
    return -(probs * torch.log(probs + 1e-10)).sum(dim=1)         # [8, B]


# ---------------------------------------------------------------- duplicate observations
_HASH_MUL = 0x100000001B3 * 0x9E37 + 1          # odd: a wrapping int64 multiply-add chain


def row_keys(x):
    """x f32 [..., C, S] -> int64 [..., S]: a hash of each column's C float bit patterns (equal
    columns -> equal keys; unequal columns may collide, group_columns verifies)."""
    bits = x.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    k = torch.zeros(bits.shape[:-2] + bits.shape[-1:], dtype=torch.int64, device=x.device)
    for c in range(bits.shape[-2]):
        k = _fmix64(k * _HASH_MUL + bits[..., c, :] + (c + 1))
    return k


GROUP_ROW = 40   # floats per sample-major feature row (38 + 2 zeros), fjsp_a2c_group_keys' rows


def group_keys(feats, rows=None):
    """feats f32 [T, 38, N] -> int64 [9, T*N]: row a < 8 = row_keys of actor a's padded inputs
    (actor_inputs), row 8 = row_keys of the critic's global state; on the GPU one pass of the
    fjsp_a2c_group_keys kernel (the same hash), which also writes each sample's features to rows
    f32 [T*N, 40] (sample-major, zero-padded: group_verify's input) when rows is given."""
    T, _, N = feats.shape
    if feats.is_cuda:
        f = feats.contiguous()
        keys = torch.empty(NA + 1, T * N, dtype=torch.int64, device=feats.device)
        if rows is not None:
            assert rows.is_contiguous() and rows.shape == (T * N, GROUP_ROW) and rows.dtype == torch.float32
        stream = torch.cuda.current_stream(feats.device).cuda_stream
        nat.check(nat.lib().fjsp_a2c_group_keys(ctypes.c_void_p(f.data_ptr()), T, N, ctypes.c_void_p(keys.data_ptr()),
                                                None if rows is None else ctypes.c_void_p(rows.data_ptr()),
                                                ctypes.c_void_p(stream)))
        return keys
    gidx = gather_index(feats.device)
    return torch.cat([row_keys(actor_inputs(feats, gidx)),
                      row_keys(feats.permute(1, 0, 2).reshape(GLOBAL_DIM, T * N))[None]])


group_buckets = True   # False: exact group counts (A/B)


def bucket(u):
    """A group count rounded up to a coarse bucket (1/16 to 1/8 of the count: ≤ 12.5 % more
    columns, ~6 % on average), so that the update's shapes (and the library kernels chosen for
    them) repeat from batch to batch.  Padding groups own no samples: computed, never gathered,
    zero gradient.  group_buckets = False: exact counts."""
    u = int(u)
    if not group_buckets or u <= 64:
        return u
    step = 1 << max(5, u.bit_length() - 4)
    return -(-u // step) * step


# the station agents' rows of a grouping of the 8 actor inputs (+ the critic's): 3 input features
# each, a few dozen distinct inputs per batch (batch_stats), grouped by the counting sort
STATION_ROWS = tuple(range(2, NA))


class RowGroups:
    """Distinct values of each row of keys int64 [R, S] (one flat sort for all rows):
    U[r] groups in row r; inv [R, S] = each sample's group, first [R, Umax] = a representative
    sample of each group (padding: any sample), rep [R, S] = the representative of each
    sample's group, perm [R, S] / ends [R, Umax] = the samples sorted by group and the end of
    each group's run (padding: S)."""

    def __init__(self, keys, lowcard=()):
        """lowcard: rows expected to hold few distinct keys (<= 64: the station agents' rows),
        grouped on the GPU by a counting sort instead of the radix sort (same result)."""
        R, S = keys.shape
        assert R <= 16, "the row id lives in bits 59..62 of the sort key"
        dev = keys.device
        if keys.is_cuda and R * S < 2 ** 31:
            self._init_device(keys, sum(1 << r for r in lowcard if r < R))
            return
        # one flat sort for all rows: the row in bits 59..62 above 59 bits of the key (the
        # grouping is verified by the caller, so a shorter key only risks a dense fallback)
        flat = (keys & ((1 << 59) - 1)) | (torch.arange(R, device=dev, dtype=torch.int64)[:, None] << 59)
        sk, fperm = torch.sort(flat.view(-1))
        sk = sk.view(R, S)
        perm = (fperm.view(R, S) - torch.arange(R, device=dev, dtype=torch.int64)[:, None] * S)
        new = torch.ones(R, S, dtype=torch.bool, device=dev)
        new[:, 1:] = sk[:, 1:] != sk[:, :-1]
        seg = _prefix_sum(new, dtype=torch.int64, add=-1).contiguous()   # each sorted position's group
        self.U = (seg[:, -1] + 1).tolist()                        # the one host sync
        umax = bucket(max(self.U))
        # each group's first sorted position (S for padding groups): a binary search of the
        # non-decreasing seg (a scatter of every position's group start sent ~10^7 stores of the
        # non-first positions to one sink column)
        starts = torch.searchsorted(seg, torch.arange(umax, device=dev).expand(R, umax).contiguous())
        self.ends = torch.cat([starts[:, 1:], torch.full((R, 1), S, dtype=torch.int64, device=dev)], 1)
        self.first = torch.gather(perm, 1, starts.clamp(max=S - 1))
        self.inv = torch.empty_like(perm).scatter_(1, perm, seg)
        self.rep = torch.gather(self.first, 1, self.inv)
        self.perm = perm
        self.gsorted = None   # the run sums' kernel input (device path only)

    def _init_device(self, keys, lowcard=0):
        """The same grouping by the library's kernels (fjsp_a2c_group_sort / _runs: one radix sort
        with 32-bit sample positions, one scan, one scatter pass; the torch path below does a 64-bit
        payload sort, a blocked prefix sum, a binary search per group and three gathers)."""
        R, S = keys.shape
        RS = R * S
        dev = keys.device
        L = nat.lib()
        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        E = lambda n, dt: torch.empty(n, dtype=dt, device=dev)  # noqa: E731
        k = keys.contiguous()
        tb = ctypes.c_uint64()
        nat.check(L.fjsp_a2c_group_temp_bytes(RS, ctypes.byref(tb)))
        temp = E(max(1, tb.value), torch.uint8)
        flat, srt = E(RS, torch.int64), E(RS, torch.int64)
        pos, spos, runs, scan = (E(RS, torch.int32) for _ in range(4))
        counts = E(R, torch.int64)
        nat.check(L.fjsp_a2c_group_sort(V(k), R, S, lowcard, V(temp), tb.value, V(flat), V(srt), V(pos), V(spos),
                                        V(runs), V(scan), V(counts), st))
        U = counts.tolist()                                       # the one host sync
        if min(U) < 0:   # a lowcard row held more than 64 distinct keys: the radix sort for every row
            nat.check(L.fjsp_a2c_group_sort(V(k), R, S, 0, V(temp), tb.value, V(flat), V(srt), V(pos), V(spos),
                                            V(runs), V(scan), V(counts), st))
            U = counts.tolist()
        del temp, flat, srt, pos, runs
        self.U = U
        umax = bucket(max(self.U))
        starts, first, ends = (E((R, umax), torch.int64) for _ in range(3))
        perm, inv, rep = (E((R, S), torch.int64) for _ in range(3))
        gsorted = E((R, S), torch.int32)
        nat.check(L.fjsp_a2c_group_runs(V(spos), V(scan), R, S, umax, V(starts), V(perm), V(inv), V(rep), V(first),
                                        V(ends), V(gsorted), st))
        self.first, self.ends, self.inv, self.rep, self.perm = first, ends, inv, rep, perm
        self.gsorted = gsorted

    def rows(self, lo, hi):
        """The groupings of rows lo..hi-1 alone (views; Umax = their own largest count)."""
        g = RowGroups.__new__(RowGroups)
        g.U = self.U[lo:hi]
        um = bucket(max(g.U))
        g.first, g.ends = self.first[lo:hi, :um], self.ends[lo:hi, :um]
        g.inv, g.perm = self.inv[lo:hi], self.perm[lo:hi]
        g.rep = None if self.rep is None else self.rep[lo:hi]
        g.gsorted = None if self.gsorted is None else self.gsorted[lo:hi]
        return g

    def gather(self, y):
        """y [R, C, Umax] per group -> [R, C, S] per sample; backward: each group's sample
        gradients summed (runs of the sorted order)."""
        return _GatherRuns.apply(y, self)


def group_columns(x, key=None):
    """Single-row RowGroups of the columns of x f32 [C, S], or None if a hash collision merged
    two different columns."""
    g = RowGroups((row_keys(x) if key is None else key)[None])
    return g if bool((x[:, g.rep[0]] == x).all()) else None


def group_verify(feats, ga, gc, x=None, gt=None, rows=None):
    """True when no hash collision merged different inputs in the groupings ga (actor inputs,
    RowGroups of group_keys rows 0..7) and gc (global states, row 8) of feats f32 [T, 38, N]:
    every sample's inputs equal those of its group's representative.  On the GPU one pass of the
    fjsp_a2c_group_verify kernel (bitwise) over rows, the sample-major rows group_keys wrote
    (made here when not given); else x [8, 13, S] / gt [38, S] compared in torch."""
    if feats.is_cuda:
        T, _, n = feats.shape
        if rows is None:
            rows = feature_rows(feats)
        bad = torch.empty(-(-(T * n) // 256), dtype=torch.int32, device=feats.device)
        stream = torch.cuda.current_stream(feats.device).cuda_stream
        V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        nat.check(nat.lib().fjsp_a2c_group_verify(V(rows), T, n, V(ga.rep), V(gc.rep), V(bad),
                                                  ctypes.c_void_p(stream)))
        return not bool(bad.any())
    ok = torch.stack([(torch.gather(x, 2, ga.rep[:, None, :].expand_as(x)) == x).all(),
                      (gt[:, gc.rep[0]] == gt).all()])
    return bool(ok.all())


class _GatherRuns(torch.autograd.Function):
    """Gather of per-group values to samples whose backward sums each group's sample gradients
    by runs of the sorted order (an f64 prefix sum differenced at the run ends): deterministic
    and free of the same-address atomic adds of index_select's backward (a station agent has
    ~10 groups for ~10^6 samples)."""

    @staticmethod
    def forward(ctx, y, g):
        ctx.g = g
        R, C, U = y.shape
        ctx.U = U
        return torch.gather(y, 2, g.inv[:, None, :].expand(R, C, g.inv.shape[1]))

    @staticmethod
    def backward(ctx, gy):
        gs = _run_sums(ctx.g, gy)                     # [R, C, Umax]: padding groups sum to 0
        if gs.shape[2] >= ctx.U:
            return gs[..., :ctx.U], None
        return torch.nn.functional.pad(gs, (0, ctx.U - gs.shape[2])), None


def _run_sums(g, gy):
    """gy [R, C, S] per sample -> [R, C, Umax] per group of the RowGroups g: runs of the sorted
    order summed (on the GPU: fjsp_a2c_run_sums, f64 sums in sorted order; else an f64 prefix sum
    differenced at the run ends)."""
    R, C, S = gy.shape
    if g.gsorted is not None:
        rowmap = _index_tensor(tuple(r for r in range(R) for _ in range(C)), gy.device).int()
        return run_sums(gy.reshape(R * C, S), rowmap, None, g).view(R, C, -1)
    ce = _prefix_at(torch.gather(gy, 2, g.perm[:, None, :].expand(R, C, S)),
                    (g.ends - 1)[:, None, :].expand(R, C, g.ends.shape[1]))
    return torch.cat([ce[..., :1], ce[..., 1:] - ce[..., :-1]], dim=-1).to(gy.dtype)


class _ActorHead(torch.autograd.Function):
    """Per-agent actor losses of A2CLosses from the agents' per-group probabilities pu [8, 8,
    Umax] (RowGroups g), computed with their per-sample gradient by one HIP kernel; backward:
    the per-sample gradients summed per group (runs of the sorted order) for the 29 valid
    (agent, action) rows only: a padded action's probability is an exact 0 out of the softmax,
    so its gradient is never used (left 0)."""

    @staticmethod
    def forward(ctx, pu, g, masks, actions, adv, adv_mean, adv_std, count, coef):
        """masks int8 [T, 29, n], actions u8 [T, 8, n], adv f64 [T, 8, n] (the slab's layouts),
        adv_mean / adv_std f32 [8] (None: the advantages as they are)."""
        T, _, n = masks.shape
        S = T * n
        grad = torch.empty(MASK_DIM, S, dtype=torch.float32, device=pu.device)
        part = torch.empty(NA, -(-S // 256), 2, dtype=torch.float64, device=pu.device)
        pu_c = pu.detach().contiguous()
        stream = torch.cuda.current_stream(pu.device).cuda_stream
        V = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
        nat.check(nat.lib().fjsp_a2c_actor_head(V(pu_c), int(pu_c.shape[2]), V(g.inv), T, n, V(masks), V(actions),
                                                V(adv), V(adv_mean), V(adv_std), 1.0 / count, coef, V(grad), V(part),
                                                ctypes.c_void_p(stream)))
        sums = part.sum(1)
        ctx.g = g
        ctx.save_for_backward(grad)
        return ((-sums[:, 0] - coef * sums[:, 1]) / count).float()

    @staticmethod
    def backward(ctx, gl):
        (grad,) = ctx.saved_tensors
        g = ctx.g
        S = grad.shape[1]
        umax = g.ends.shape[1]
        if g.gsorted is not None:   # the device grouping: one run-sum pass (fjsp_a2c_run_sums)
            row_agent = _index_tensor(tuple(a for a in range(NA) for _ in range(N_ACTIONS[a])), grad.device)
            rs = run_sums(grad, row_agent, gl.to(grad.dtype)[row_agent], g)              # [29, Umax]
            out = torch.zeros(NA * 8, umax, dtype=grad.dtype, device=grad.device)
            out[_valid_rows(grad.device)] = rs
            return out.view(NA, 8, umax), None, None, None, None, None, None, None, None
        # each agent's rows in its sorted sample order, scaled by the agent's loss gradient
        srt = torch.empty_like(grad)
        for a in range(NA):
            o, k = MASK_OFFS[a], N_ACTIONS[a]
            torch.gather(grad[o:o + k], 1, g.perm[a].expand(k, S), out=srt[o:o + k])
        row_agent = _index_tensor(tuple(a for a in range(NA) for _ in range(N_ACTIONS[a])), grad.device)
        srt.mul_(gl.to(grad.dtype)[row_agent, None])
        ce = _prefix_at(srt, (g.ends - 1)[row_agent])
        rs = torch.cat([ce[:, :1], ce[:, 1:] - ce[:, :-1]], dim=1).to(grad.dtype)    # [29, Umax]
        out = torch.zeros(NA * 8, umax, dtype=grad.dtype, device=grad.device)
        out[_valid_rows(grad.device)] = rs
        return out.view(NA, 8, umax), None, None, None, None, None, None, None, None


_VALID_ROWS = {}
_INDEX = {}


def _index_tensor(values, device):
    """A small int64 index tensor on `device`, built once per (values, device): a host-to-device
    copy must not happen inside a graph capture (the captured update, VecMultiAgentA2C)."""
    key = (values, torch.device(device))
    if key not in _INDEX:
        _INDEX[key] = torch.tensor(values, dtype=torch.int64, device=device)
    return _INDEX[key]


def warm_index_tensors(device):
    """Every index tensor the grouped update may ask for (each choice of the largest actor)."""
    for big in range(NA):
        _index_tensor(tuple(a for a in range(NA) if a != big), device)
        _index_tensor((big,), device)
    _index_tensor(tuple(a for a in range(NA) for _ in range(N_ACTIONS[a])), device)
    _valid_rows(device)


def _valid_rows(device):
    """Rows a * 8 + j (j < N_ACTIONS[a]) of [8 * 8, .]: the 29 valid (agent, action) pairs in
    action-mask order."""
    if device not in _VALID_ROWS:
        _VALID_ROWS[device] = torch.tensor([a * 8 + j for a in range(NA) for j in range(N_ACTIONS[a])],
                                           device=device)
    return _VALID_ROWS[device]


def run_sums(vals, rowmap, scale, g):
    """out [J, Umax] f32: per group of row rowmap[j] of the (device) RowGroups g, the f64 sum in
    sorted order of vals[j] (* scale[j]) over the group's samples (fjsp_a2c_run_sums)."""
    J, S = vals.shape
    umax = g.first.shape[1]
    dev = vals.device
    v = vals.contiguous()
    rm = rowmap.to(torch.int32).contiguous()
    sc = None if scale is None else scale.to(torch.float32).contiguous()
    tb = ctypes.c_uint64()
    nat.check(nat.lib().fjsp_a2c_run_sums_bytes(J, S, ctypes.byref(tb)))
    temp = torch.empty(tb.value, dtype=torch.uint8, device=dev)
    out = torch.empty(J, umax, dtype=torch.float32, device=dev)
    perm, gs = g.perm.contiguous(), g.gsorted.contiguous()
    V = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
    nat.check(nat.lib().fjsp_a2c_run_sums(V(v), J, V(rm), V(sc), V(perm), V(gs), S, umax, V(temp), tb.value, V(out),
                                          ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    return out


def _prefix_at(w, idx, block=1024):
    """The f64 inclusive prefix sums of w [..., S] along the last dim at positions idx [..., K]
    only: _prefix_sum(w.double()) gathered at idx, bit for bit (the same block scans, the same
    block offsets added), without casting w to f64 in a pass of its own (the scan casts) or
    adding the block offsets to all S sums (only the K gathered ones)."""
    *lead, S = w.shape
    P = -(-S // block) * block
    wp = w if P == S else torch.nn.functional.pad(w, (0, P - S))
    c = wp.reshape(*lead, P // block, block).cumsum(-1, dtype=torch.float64)
    tot = c[..., -1]
    off = tot.cumsum(-1) - tot                                   # exclusive block offsets
    return torch.gather(c.view(*lead, P), -1, idx) + torch.gather(off, -1, idx // block)


def _prefix_sum(w, block=1024, dtype=None, add=0):
    """Inclusive prefix sum along the last dim (in dtype, + add), blocked so every scan runs over
    many short rows (a scan over a few 10^6-long rows is one slow row per row)."""
    *lead, S = w.shape
    P = -(-S // block) * block
    wp = w if P == S else torch.nn.functional.pad(w if dtype is None else w.to(dtype), (0, P - S))
    c = wp.reshape(*lead, P // block, block).cumsum(-1, dtype=dtype)
    tot = c[..., -1]
    off = tot.cumsum(-1) - tot
    if add:
        off = off + add
    c = c + off[..., None]
    return c.view(*lead, P)[..., :S]


class A2CLosses:
    """Loss sums for one (possibly sharded) batch; `count` = the GLOBAL sample count.

    actor_loss_a = -(mean(adv_n * logp)) - c * mean(entropy) where adv_n uses the global
    mean / unbiased std of agent a's advantages (calc_actor_loss, a2c.py:724-731); critic =
    mean over (agent, sample) of (V - R)^2 (calc_critic_loss, a2c.py:713-722).  With shards,
    every rank passes the global statistics and count, so summing the per-rank gradients
    (all_reduce) gives the single-learner gradient.

    dedup: every network runs once per DISTINCT input of the batch and its outputs are gathered
    per sample.  An agent's observation repeats across steps and envs (in a 256 x 1024
    masked-random batch the six station agents see <= 28 distinct observations, the pickup
    station 1 225, the AGV 16 % of the samples, the critic's global state 75 %).  The losses
    are built from the gathered outputs exactly as without dedup, so the gather's backward sums
    each sample's gradient into its distinct input: the same gradient, summed in another order."""

    @staticmethod
    def compute(actors, critic, feats, masks, actions, returns, adv, gidx, midx, entropy_coef,
                adv_mean, adv_std, count, dedup=False, groups=None):
        """The rollout slab's layouts: feats f32 [T, 38, N], masks int8 [T, 29, N], actions u8
        [T, 8, N], returns / adv f64 [T, 8, N] (a single step may drop the T axis).  groups =
        (ga, gc): a verified grouping computed by the caller; else dedup groups here (keys, sort,
        check: two host synchronisations).  On the GPU the grouped path's loss head reads actions
        and advantages in the slab layouts; [8, S] copies are made for the dense / CPU path only."""
        f3 = feats if feats.dim() == 3 else feats[None]
        m3 = masks if masks.dim() == 3 else masks[None]
        a3 = actions if actions.dim() == 3 else actions[None]
        r3 = returns if returns.dim() == 3 else returns[None]
        d3 = adv if adv.dim() == 3 else adv[None]
        T, _, n = f3.shape
        S = T * n
        ga = gc = None
        rows = None
        if groups is not None:
            ga, gc = groups
        elif dedup:
            f3 = f3.contiguous()
            rows = torch.empty(S, GROUP_ROW, dtype=torch.float32, device=f3.device) if f3.is_cuda else None
            gr = RowGroups(group_keys(f3, rows), STATION_ROWS)      # 8 actor rows + the critic's
            ga, gc = gr.rows(0, NA), gr.rows(NA, NA + 1)
            x = gv = None
            if not feats.is_cuda:
                x, gv = actor_inputs(feats, gidx), f3.permute(1, 0, 2).reshape(GLOBAL_DIM, S)
            if not group_verify(f3, ga, gc, x, gv, rows):           # a hash collision: dense
                ga = gc = None

        if ga is not None and feats.is_cuda:
            # the groups' representatives gathered as whole sample-major rows (160 B each) of the
            # keys pass's rows: no [38, S] copy of the slab, no 38 scattered words per column
            if rows is None:
                rows = feature_rows(f3)

            def cols(agents, idx):                                   # [k, 13, u]
                k, u = idx.shape
                r = rows.index_select(0, idx.reshape(-1)).view(k, u, GROUP_ROW)
                return torch.gather(r, 2, gidx[agents][:, None, :].expand(k, u, gidx.shape[1])).transpose(1, 2)
        else:
            # the global states as feature rows [38, S]: one copy of the slab, then row-wise
            # gathers of the groups' representatives
            gt = f3.permute(1, 0, 2).reshape(GLOBAL_DIM, S)

            def cols(agents, idx):                                   # [k, 13, u] from gt
                k, u = idx.shape
                c = gt[:, idx.reshape(-1)].view(GLOBAL_DIM, k, u)
                c = torch.cat([c, c.new_zeros(1, k, u)])
                return c[gidx[agents], torch.arange(k, device=idx.device)[:, None], :]
        # the critic first: its GEMMs keep the GPU busy while the host issues the actors' many
        # small launches (after the grouping's host synchronisations the queue is empty)
        critic_loss = None
        if gc is not None and feats.is_cuda and critic_fused and critic_onepass_on and gc.gsorted is not None:
            critic_loss = critic_onepass(critic, rows.index_select(0, gc.first[0]), critic_coef(gc, r3, count))
            v = None
        elif gc is not None and feats.is_cuda and gc.first.shape[1] >= 65536 and critic_fused:
            vu = critic_grouped(critic, rows.index_select(0, gc.first[0])).reshape(1, 1, -1)
            v = gc.gather(vu).reshape(-1)                            # [S]
        elif gc is not None and feats.is_cuda:
            vu = mlp_forward(critic.net, rows.index_select(0, gc.first[0])[:, :GLOBAL_DIM]).reshape(1, 1, -1)
            v = gc.gather(vu).reshape(-1)                            # [S]
        elif gc is not None:
            vu = mlp_forward(critic.net, gt[:, gc.first[0]].t()).reshape(1, 1, -1)
            v = gc.gather(vu).reshape(-1)                            # [S]
        else:
            v = mlp_forward(critic.net, gt.t()).reshape(-1)
        norm = count > 1
        if ga is not None and feats.is_cuda:
            # the loss head and its gradient in one kernel (fjsp_a2c_actor_head), on the slabs
            actor_losses = _ActorHead.apply(actors.forward_rows(None, ga, cols), ga, m3.contiguous(), a3.contiguous(),
                                            d3.contiguous(), adv_mean if norm else None, adv_std if norm else None,
                                            float(count), float(entropy_coef))
        else:
            x = actor_inputs(feats, gidx)                            # [8, 13, S]
            acts = a3.long().permute(1, 0, 2).reshape(NA, S)
            adv32 = d3.float().permute(1, 0, 2).reshape(NA, S)        # calc_actor_loss: FloatTensor(adv)
            adv_n = (adv32 - adv_mean[:, None]) / (adv_std[:, None] + 1e-8) if norm else adv32
            if ga is not None:
                probs = ga.gather(actors.forward_rows(x, ga, cols))  # [8, 8, S]
            else:
                probs = actors(x)                                    # [8, 8, S]
            ent = entropy_of(probs)                                  # [8, S]
            pm = masked_probs(probs, agent_masks(masks, midx))
            logp = categorical_log_prob(pm, acts)                    # [8, S]
            actor_losses = -(adv_n * logp).sum(dim=1) / count - entropy_coef * ent.sum(dim=1) / count
        if critic_loss is None:
            critic_loss = ((v.view(T, 1, n) - r3.float()) ** 2).sum() / (NA * count)
        return actor_losses, critic_loss


def clip_per_agent_(actors, max_norm):
    """torch.nn.utils.clip_grad_norm_ applied to each agent's actor separately (a2c.py:675-679)."""
    grads = [p.grad for p in actors.parameters() if p.grad is not None]
    # every agent's gradients as one row, one norm launch (was three launches per parameter)
    norm = torch.linalg.vector_norm(torch.cat([g.reshape(NA, -1) for g in grads], dim=1), dim=1)
    coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
    for g in grads:
        g.mul_(coef.view(NA, *([1] * (g.dim() - 1))))
    return norm


# ---------------------------------------------------------------- fused policy kernel weights
def split_bf16x3(W):
    """f32 -> (hi, mid, lo) bf16 with W = hi + mid + lo up to 2^-24 |W| (each difference is exact
    in f32; round to nearest even, as the kernel splits its activations)."""
    W = W.float()
    hi = W.to(torch.bfloat16)
    r = W - hi.float()
    mid = r.to(torch.bfloat16)
    return hi, mid, (r - mid.float()).to(torch.bfloat16)


def pack_mfma(W):
    """[..., R, K] f32 -> [..., R/32, K/16, 3, 64, 4] f32 words holding [..., 3, 64, 8] bf16 with
    (t, kb, p, l, j) = plane p of W[32 t + (l & 31)][16 kb + 8 (l >> 5) + j]: the A-operand lane order
    of v_mfma_f32_32x32x16_bf16, one 16-byte load per lane per plane and 16-deep block, the three
    planes of split_bf16x3 (csrc/fjsp_policy.hip, include/fjsp.h).  On the GPU one launch of
    fjsp_a2c_pack_mfma (bit-equal to the torch formulation below); W may be a transposed view of
    a contiguous [..., K, R] tensor."""
    *lead, R, K = W.shape
    if W.is_cuda and W.dtype == torch.float32 and R % 32 == 0 and K % 16 == 0 and pack_kernel_on:
        B = 1
        for d in lead:
            B *= d
        tr = 0
        src = W
        if not W.is_contiguous():
            if W.dim() >= 2 and W.transpose(-1, -2).is_contiguous():
                src, tr = W.transpose(-1, -2), 1
            else:
                src = W.contiguous()
        out = torch.empty(*lead, R // 32, K // 16, 3, 64, 4, dtype=torch.float32, device=W.device)
        nat.check(nat.lib().fjsp_a2c_pack_mfma(ctypes.c_void_p(src.data_ptr()), B, R, K, tr,
                                               ctypes.c_void_p(out.data_ptr()),
                                               ctypes.c_void_p(torch.cuda.current_stream(W.device).cuda_stream)))
        return out
    return pack_mfma_torch(W)


pack_kernel_on = True   # False: the weight packing in torch ops (A/B)


def pack_mfma_torch(W):
    """pack_mfma in torch ops (CPU, and the GPU test's reference)."""
    *lead, R, K = W.shape
    nl = len(lead)
    Pl = torch.stack(split_bf16x3(W), dim=nl)                                # [..., 3, R, K]
    Pl = Pl.reshape(*lead, 3, R // 32, 32, K // 16, 2, 8)                     # p, t, i, kb, hh, j
    Pl = Pl.permute(*range(nl), nl + 1, nl + 3, nl, nl + 4, nl + 2, nl + 5)   # t, kb, p, hh, i, j
    return Pl.contiguous().view(torch.float32).reshape(*lead, R // 32, K // 16, 3, 64, 4)


@torch.no_grad()
def pack_critic_weights(W1, b1, W2, b2, W3, b3, W4, b4):
    """The critic's layers (networks.CentralizedCriticNetwork: 38 -> 256 -> 256 -> 128 -> 1) -> the
    flat buffer fjsp_a2c_policy / fjsp_a2c_critic_forward read (include/fjsp.h)."""
    z = W1.new_zeros
    w1 = torch.cat([W1, z(W1.shape[0], nat.POLICY_CRITIC_DPAD - W1.shape[1])], dim=1)   # [256, 48]
    return torch.cat([pack_mfma(w1).reshape(-1), b1.reshape(-1), pack_mfma(W2).reshape(-1), b2.reshape(-1),
                      pack_mfma(W3).reshape(-1), b3.reshape(-1), W4.reshape(-1), torch.cat([b4.reshape(-1), z(15)])])


@torch.no_grad()
def pack_policy_weights(actors, critic, out_actor=None, out_critic=None):
    """Actor stack + critic -> the flat buffers fjsp_a2c_policy reads (include/fjsp.h): the MFMA
    layers' weights as bf16 planes in lane order, biases and the VALU layers as f32."""
    dev = actors.W1.device
    z = lambda *s: torch.zeros(*s, device=dev)  # noqa: E731
    w1 = torch.cat([actors.W1, z(NA, actors.hidden, nat.POLICY_ACTOR_DPAD - DPAD)], dim=2)   # [8, 256, 16]
    b3 = torch.cat([actors.b3[:, :, 0], z(NA, 8)], dim=1)                                     # [8, 16]
    a = torch.cat([pack_mfma(w1).reshape(NA, -1), actors.b1.reshape(NA, -1), pack_mfma(actors.W2).reshape(NA, -1),
                   actors.b2.reshape(NA, -1), actors.W3.reshape(NA, -1), b3], dim=1).reshape(-1)
    c = pack_critic_weights(*[m for i in (0, 2, 4, 6) for m in (critic.net[i].weight, critic.net[i].bias)])
    assert a.numel() == NA * nat.POLICY_ACTOR_FLOATS and c.numel() == nat.POLICY_CRITIC_FLOATS
    if out_actor is None:
        return a.contiguous(), c.contiguous()
    out_actor.copy_(a)
    out_critic.copy_(c)
    return out_actor, out_critic


def init_networks(seed=None, hidden=256, device="cpu"):
    """Actor stack + critic initialised exactly like MultiAgentA2C.__init__ (a2c.py:87-103):
    the 8 ActorNetworks in possible_agents order, then the critic, from torch's CPU generator
    (torch.manual_seed(seed) first when seed is given), then moved to `device`."""
    if seed is not None:
        torch.manual_seed(seed)
    nets = [ActorNet(OBS_DIMS[a], N_ACTIONS[a], hidden) for a in range(NA)]
    critic = CriticNet(GLOBAL_DIM, hidden)
    actors = ActorStack(hidden)
    actors.load_actor_nets(nets)
    return actors.to(device), critic.to(device)


def flat_grads(actors, critic):
    """Every parameter's gradient (8 stacked actors, then the critic) as one flat f32 tensor."""
    return torch.cat([p.grad.reshape(-1) if p.grad is not None else torch.zeros_like(p).reshape(-1)
                      for p in list(actors.parameters()) + list(critic.parameters())])


def update_core(actors, critic, optim_actor, optim_critic, feats, masks, actions, ret, adv, gidx, midx,
                entropy_coef, max_grad_norm, group=None, dedup=False, grad_probe=None, groups=None):
    """update_step without the final host copies: returns the (all-reduced) actor losses [8] and
    critic loss [1] as device tensors.  With groups (a verified grouping) and no group / probe it
    issues no host synchronisation, so a graph can capture it."""
    from . import distributed as D
    count, mean, std = D.adv_stats_slab(adv, group)                  # of FloatTensor(adv), a2c.py:724-731
    optim_actor.zero_grad(set_to_none=True)
    optim_critic.zero_grad(set_to_none=True)
    actor_losses, critic_loss = A2CLosses.compute(actors, critic, feats, masks, actions, ret, adv, gidx, midx,
                                                  entropy_coef, mean, std, count, dedup, groups)
    (actor_losses.sum() + critic_loss).backward()
    D.allreduce_grads(list(actors.parameters()) + list(critic.parameters()), group)
    if grad_probe is not None:
        grad_probe(flat_grads(actors, critic).detach().clone())
    clip_per_agent_(actors, max_grad_norm)
    torch.nn.utils.clip_grad_norm_(critic.parameters(), max_grad_norm)
    optim_actor.step()
    optim_critic.step()
    al = D.allreduce_sum(actor_losses.detach(), group)
    cl = D.allreduce_sum(critic_loss.detach().view(1), group)
    return al, cl


def update_step(actors, critic, optim_actor, optim_critic, feats, masks, actions, ret, adv, gidx, midx,
                entropy_coef, max_grad_norm, group=None, dedup=False, grad_probe=None):
    """One _update (a2c.py:647-703) on a [T, ., N] batch (this rank's shard of it).

    feats f32 [T, 38, N], masks int8 [T, 29, N], actions u8 [T, 8, N], ret / adv f64 [T, 8, N].
    grad_probe(flat f32 grads): called with the reduced gradients before clipping and Adam
    (tests compare them across exchanges).
    Returns (actor losses per agent, critic loss) as Python floats (the loss histories)."""
    al, cl = update_core(actors, critic, optim_actor, optim_critic, feats, masks, actions, ret, adv, gidx, midx,
                         entropy_coef, max_grad_norm, group, dedup, grad_probe)
    return al.cpu().tolist(), float(cl.cpu()[0])


def batch_advantages(rewards, values, done, gamma, lamb, use_gae=True):
    """finish_trajectory (transition_memory.py:45-105) over a [T, ., N] batch with the fp64
    GAE kernel.  rewards f64 [T, 8, N], values f32 [T + 1, N] (row T = V(s_T), the batch-end
    bootstrap, a2c.py:321-332), done u8/bool [T, N] (an episode end bootstraps 0, a2c.py:357).
    Returns ret, adv f64 [T, 8, N]."""
    from .vec_env import gae_shared
    T, _, N = rewards.shape
    ret, adv = gae_shared(rewards, values, done, gamma, lamb)
    if not use_gae:
        adv = ret - values[:T, None, :].double()
    return ret, adv


class VecMultiAgentA2C:
    """MultiAgentA2C for an FJSPVecEnv (N envs on this GPU; optionally one shard of a
    multi-GPU job through `group`).

    Hyper-parameters and their defaults follow train.py:57-98 (batch 256, gamma 0.99,
    lambda 0.95, lr 3e-4 / 1e-3, entropy 0.01, clip 0.5)."""

    def __init__(self, env, batch_size=256, gamma=0.99, lamb=0.95, lr_actor=3e-4, lr_critic=1e-3,
                 use_gae=True, entropy_coef=0.01, max_grad_norm=0.5, hidden=256, seed=None, group=None,
                 use_graph=None, fused_policy=True, exchange="allreduce", dedup=True):
        self.env = env
        self.device = env.device
        self.N = env.num_envs
        self.batch_size = int(batch_size)
        self.gamma, self.lamb = float(gamma), float(lamb)
        self.use_gae = use_gae
        self.entropy_coef = float(entropy_coef)
        self.max_grad_norm = float(max_grad_norm)
        self.group = group
        if exchange not in ("allreduce", "gather", "shard"):
            raise ValueError("exchange must be 'allreduce', 'gather' or 'shard'")
        self.exchange = exchange
        self.dedup = bool(dedup)   # networks once per distinct input in the update (A2CLosses)
        self.possible_agents = list(AGENTS)
        self.obs_dims = dict(zip(AGENTS, OBS_DIMS))
        self.act_dims = dict(zip(AGENTS, N_ACTIONS))
        self.global_obs_dim = GLOBAL_DIM
        self.actors, self.critic = init_networks(seed, hidden, self.device)
        fused = self.device.type == "cuda"      # one multi-tensor kernel per step (same Adam math)
        # capturable: the step counters live on the device, so the update can be graph-captured
        self.optim_actor = torch.optim.Adam(self.actors.parameters(), lr=lr_actor, fused=fused, capturable=fused)
        self.optim_critic = torch.optim.Adam(self.critic.parameters(), lr=lr_critic, fused=fused, capturable=fused)
        self.gidx = gather_index(self.device)
        self.midx = mask_index(self.device)
        self.actor_loss_history = {a: [] for a in AGENTS}
        self.critic_loss_history = []
        self.episode_end_timesteps = []
        self._bufs = None
        # None: decided per collect (_graph_on); True / False: always / never replay a captured graph
        self.use_graph = None if use_graph is None else bool(use_graph) and self.device.type == "cuda"
        # fused policy kernel (csrc/fjsp_policy.hip): one launch per vector step
        self.fused_policy = bool(fused_policy) and self.device.type == "cuda" and hidden == 256
        # ... with the env step inside the same launch (fjsp_a2c_policy_step; False: the policy
        # kernel, then fjsp_step, two launches per vector step, the same bytes)
        self.fused_step = self.fused_policy
        # env groups of the fused collect, each on a stream of its own (_collect_groups)
        self.collect_groups = 2
        self._streams = None
        self._collect_values = True        # diagnostics: False = the collect without the critic
        # sampling key: (seed, batch) -> counter hash per (global env id, step, agent); the same
        # on every rank, the env's global id separates the shards
        self._rng_host = int.from_bytes(__import__("os").urandom(7), "little") if seed is None else int(seed)
        # the draw key lives on the device for both policy paths: a captured collect reads it
        # at replay time, so every replay draws new actions
        self._rng = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._rng.fill_(_s64(self._rng_host))   # the kernel's uint64 key, wrapped to int64
        role_keys(self.device)
        if self.fused_policy:
            self._pw_actor, self._pw_critic = pack_policy_weights(self.actors, self.critic)
        self._graph = None
        self._graph_det = None
        self._eager_batches = 0
        self.gae_fn = batch_advantages     # finish_trajectory over a batch (tests may inject a CPU stand-in)
        self.grad_probe = None             # grad_probe(flat reduced grads) before clip / Adam (tests)
        self.exchange_timing = None        # dict of synchronised stage times (ms) when not None (bench)
        self.shard_info = {}               # exchange="shard": the last batch's record counts and bytes

    # ------------------------------------------------------------ rollout storage
    def _alloc(self):
        T, N, dev = self.batch_size, self.N, self.device
        z = lambda *s, dt: torch.zeros(*s, dtype=dt, device=dev)  # noqa: E731
        b = {
            "feats": z(T + 1, GLOBAL_DIM, N, dt=torch.float32),
            "masks": z(T + 1, 29, N, dt=torch.int8),
            "actions": z(T, NA, N, dt=torch.uint8),
            "values": z(T + 1, N, dt=torch.float32),
            "rewards": z(T, NA, N, dt=torch.float64),
            "term": z(T, N, dt=torch.uint8),
            "trunc": z(T, N, dt=torch.uint8),
            "status": z(T, N, dt=torch.int32),
        }
        outs = []
        for t in range(T):
            o = nat.fjsp_out()
            o.rewards = b["rewards"][t].data_ptr()
            o.term = b["term"][t].data_ptr()
            o.trunc = b["trunc"][t].data_ptr()
            o.status = b["status"][t].data_ptr()
            o.next_masks = b["masks"][t + 1].data_ptr()
            o.feats = b["feats"][t + 1].data_ptr()
            outs.append(o)
        b["outs"] = outs
        self._bufs = b

    def reset(self, seeds=None, num_orders=25):
        """env.reset + the first observation's features (a2c.py:269)."""
        if self._bufs is None:
            self._alloc()
        b = self._bufs
        o = nat.fjsp_out()
        o.masks = b["masks"][0].data_ptr()
        o.feats = b["feats"][0].data_ptr()
        self.env._sync_stream()
        if seeds is None and getattr(self.env, "_pending_seeds", None) is not None:
            seeds = self.env._pending_seeds   # FJSPVecEnv.seed(...) before the learner's reset
        self.env._pending_seeds = None
        s = None
        if seeds is not None:
            s = torch.as_tensor(seeds, device=self.device).to(torch.int64).bitwise_and(0xFFFFFFFF).to(torch.int32)
        nat.check(nat.lib().fjsp_reset(self.env.handle, None if s is None else ctypes.c_void_p(s.data_ptr()),
                                       None, int(num_orders), ctypes.byref(o)))
        self.num_orders = int(num_orders)

    # ------------------------------------------------------------ predict
    @torch.no_grad()
    def policy_fused(self, feats, masks, t, deterministic, act_out, val_out, probs_out=None, gid0=None):
        """fjsp_a2c_policy on this stream: actions u8 [8, N] -> act_out, values -> val_out."""
        stream = torch.cuda.current_stream(self.device).cuda_stream
        P = lambda x: None if x is None else ctypes.c_void_p(x.data_ptr())  # noqa: E731
        rc = nat.lib().fjsp_a2c_policy(P(feats), P(masks), int(feats.shape[-1]), P(self._pw_actor),
                                       P(self._pw_critic), P(self._rng), int(gid0 if gid0 is not None else
                                                                                self.env.env_id_base),
                                       int(t), int(bool(deterministic)),
                                       P(act_out), P(val_out), P(probs_out), ctypes.c_void_p(stream))
        nat.check(rc)

    def policy_step(self, t, deterministic, env_begin=0, env_count=None, stream=None):
        """Vector step t of the collect in one launch (fjsp_a2c_policy_step): the fused policy's
        actions and values, then the env step of each 64-env tile by its last actor workgroup,
        writing rewards / term / trunc / status and the next observation's masks and features into
        the rollout slab (bytes equal to policy_fused + fjsp_step).  env_begin / env_count: the
        envs of this launch (whole 64-env tiles), on `stream` (default: the current stream)."""
        b = self._bufs
        P = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
        st = (stream or torch.cuda.current_stream(self.device)).cuda_stream
        nat.check(nat.lib().fjsp_a2c_policy_step(self.env.handle, P(b["feats"][t]), P(b["masks"][t]), P(self._pw_actor),
                                                 P(self._pw_critic), P(self._rng), int(self.env.env_id_base), int(t),
                                                 int(bool(deterministic)), P(b["actions"][t]),
                                                 P(b["values"][t]) if self._collect_values else None, 1,
                                                 ctypes.byref(b["outs"][t]), int(env_begin),
                                                 int(self.N - env_begin if env_count is None else env_count),
                                                 ctypes.c_void_p(st)))

    def _collect_groups(self):
        """The collect's env groups: (env_begin, env_count) of whole 64-env tiles, collect_groups of
        them (fewer when N has fewer tiles).  Each group's chain of vector steps runs on a stream of
        its own: the groups' launches overlap, so one group's env-step tail runs beside another's
        network layers (the step's chain needs only its own tiles)."""
        tiles = -(-self.N // 64)
        g = max(1, min(int(self.collect_groups), tiles))
        out, t0 = [], 0
        for i in range(g):
            nt = tiles // g + (1 if i < tiles % g else 0)
            e0, e1 = 64 * t0, min(self.N, 64 * (t0 + nt))
            out.append((e0, e1 - e0))
            t0 += nt
        return out

    def repack(self):
        """Refresh the fused kernel's packed weights (after an update / load)."""
        if self.fused_policy:
            pack_policy_weights(self.actors, self.critic, self._pw_actor, self._pw_critic)

    @torch.no_grad()
    def policy(self, feats, masks, deterministic=False, t=0, gid0=None):
        """predict (a2c.py:168-252) for all agents and envs: actions long [8, B], the masked
        probabilities [8, 8, B] and the critic's value [B].  Draws use the fused kernel's
        counter hash keyed by (seed, global env id, t, agent)."""
        pm = masked_probs(self.actors(actor_inputs(feats, self.gidx)), agent_masks(masks, self.midx))
        if deterministic:
            act = torch.argmax(pm, dim=1)
        else:
            g0 = self.env.env_id_base if gid0 is None else gid0
            gid = torch.arange(g0, g0 + pm.shape[2], device=pm.device)
            act = sample_categorical(pm, counter_uniform(self._rng, gid, t, pm.device))
        v = self.critic(feats.t()).view(-1)
        return act, pm, v

    def predict(self, feats, masks, deterministic=False, train_returns=False):
        """Actions u8 [8, B] (+ log-probs [8, B] and values [B] with train_returns)."""
        act, pm, v = self.policy(feats, masks, deterministic)
        if train_returns:
            return act.to(torch.uint8), categorical_log_prob(pm, act), v
        return act.to(torch.uint8)

    # ------------------------------------------------------------ one batch
    def collect(self, deterministic=False, action_fn=None):
        """batch_size vector steps: predict -> fjsp_step (features + masks of the next
        observation written in place) -> memory.  action_fn(t, masks) may override actions
        (tests).  After one eager batch the whole batch (batch_size x (policy + step) plus the
        bootstrap value, ~40 launches per step) is captured once into a hipGraph and replayed:
        the buffers and parameters are static, Adam updates the weights in place."""
        self._rng_host += 1
        self._rng.fill_(_s64(self._rng_host))   # re-keys the sampling of the (captured) batch
        if action_fn is None and self._graph_on():
            if self._graph is not None and self._graph_det == deterministic:
                self._graph.replay()
                return
            if self._eager_batches >= 1:
                self._capture(deterministic)
                self._graph.replay()
                return
        self._collect_eager(deterministic, action_fn)
        self._eager_batches += 1

    def _graph_on(self):
        """use_graph None (the default): replay a captured graph of the batch, except for the fused
        collect on two or more env-group streams, whose launches are issued eagerly: the groups'
        step chains then overlap more than in the graph's replay (collect 6.2-6.5 against 6.8-7.1 ms
        per 256 x 4 096 batch, slabs byte-equal; profiles/r06/a2c/collect_graph_ab.json), and one
        launch per group and step keeps the host ahead of the GPU."""
        if self.use_graph is not None:
            return self.use_graph
        return self.device.type == "cuda" and not (self.fused_step and len(self._collect_groups()) >= 2)

    def _capture(self, deterministic):
        L = nat.lib()
        h = self.env.handle
        nat.check(L.fjsp_set_option(h, b"timing", 0))   # no hipEventRecord inside the capture
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g):
                self._collect_eager(deterministic, None)
        finally:
            self.env._sync_stream()
            nat.check(L.fjsp_set_option(h, b"timing", 1))
        self._graph, self._graph_det = g, deterministic

    def _collect_eager(self, deterministic, action_fn):
        b = self._bufs
        L = nat.lib()
        h = self.env.handle
        self.env._sync_stream()
        T = self.batch_size
        if self.fused_step and action_fn is None:
            groups = self._collect_groups()
            if len(groups) == 1:
                for t in range(T):
                    self.policy_step(t, deterministic)
            else:
                cur = torch.cuda.current_stream(self.device)
                if self._streams is None or len(self._streams) != len(groups):
                    self._streams = [torch.cuda.Stream(self.device) for _ in groups]
                for s in self._streams:
                    s.wait_stream(cur)
                for t in range(T):
                    for (e0, cnt), s in zip(groups, self._streams):
                        self.policy_step(t, deterministic, e0, cnt, s)
                for s in self._streams:
                    cur.wait_stream(s)
        for t in range(0 if self.fused_step and action_fn is None else T):
            if self.fused_policy and action_fn is None:
                self.policy_fused(b["feats"][t], b["masks"][t], t, deterministic, b["actions"][t], b["values"][t])
            else:
                act, _, v = self.policy(b["feats"][t], b["masks"][t], deterministic, t=t)
                if action_fn is not None:
                    act = action_fn(t, b["masks"][t]).to(self.device).long()
                b["actions"][t].copy_(act)
                b["values"][t].copy_(v)
            nat.check(L.fjsp_step(h, ctypes.c_void_p(b["actions"][t].data_ptr()), None, 1,
                                  ctypes.byref(b["outs"][t])))
        with torch.no_grad():
            if self.fused_policy:
                # the bootstrap V(s_T) by the same kernel as every step's value: a value depends
                # only on its env's features, never on how the envs are sharded
                self.policy_fused(b["feats"][T], None, T, True, None, b["values"][T])
            else:
                b["values"][T].copy_(self.critic(b["feats"][T].t()).view(-1))

    def advantages(self):
        """finish_trajectory over the batch (transition_memory.py:45-105) with the fp64 GAE
        kernel: an episode end bootstraps 0 (a2c.py:357), the batch end V(s_T) (a2c.py:321-332)."""
        b = self._bufs
        return self.gae_fn(b["rewards"], b["values"], b["term"] | b["trunc"], self.gamma, self.lamb, self.use_gae)

    def _start(self):
        """Start of a timed stage sequence (synchronises when exchange_timing is on, so the
        previous work, e.g. the collect's graph replay, is not counted)."""
        import time
        if self.exchange_timing is not None and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        return time.perf_counter()

    def _mark(self, name, t0):
        """Stage timing for the bench (synchronising): adds ms since t0 to exchange_timing."""
        import time
        if self.exchange_timing is None:
            return t0
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        t = time.perf_counter()
        self.exchange_timing[name] = self.exchange_timing.get(name, 0.0) + (t - t0) * 1e3
        return t

    def update(self, ret=None, adv=None):
        """_update (a2c.py:647-703) over the batch's T x N transitions (x world with a group).

        exchange "allreduce": GAE on this rank, one flat gradient all_reduce (distributed.py);
        exchange "gather": the transitions go to the learner rank (ret / adv are recomputed
        there over the gathered batch), the new parameters come back in one broadcast.  Only
        the learner rank steps Adam under "gather": its moments live there (the other ranks'
        optimisers stay at their initial state), so a run that later switches to "allreduce"
        or resumes an optimiser must take it from the learner rank."""
        from . import distributed as D
        # synchronises; the update has host syncs of its own.  With several ranks the fault words
        # are max-reduced first, so every rank raises together instead of the healthy ones
        # waiting in the exchange for one that raised
        fw = D.max_over_ranks(self.env.faults(), self.group, self.device)
        if fw:
            raise RuntimeError(f"fjsp step kernels reported fault word {fw:#x} (a hand-off wait gave up): "
                               "the batch's transitions are invalid")
        if self.exchange == "gather" and D.active(self.group):
            al, cl = self._update_gathered()
        elif self.exchange == "shard" and D.active(self.group):
            from . import shard_learner as SL
            t0 = self._start()
            if ret is None:
                ret, adv = self.advantages()
            b = self._bufs
            T = self.batch_size
            info = {}
            stage = None
            if self.exchange_timing is not None:   # the bench's stats batch: every stage synchronised
                clock = [self._mark("shard_gae", t0)]

                def stage(name):
                    clock[0] = self._mark("shard_" + name, clock[0])
            al, cl = SL.update_sharded(self.actors, self.critic, self.optim_actor, self.optim_critic, b["feats"][:T],
                                       b["masks"][:T], b["actions"], ret, adv, self.gidx, self.midx, self.entropy_coef,
                                       self.max_grad_norm, self.group, self.dedup, self.grad_probe, info, stage)
            self.shard_info = info
            self._mark("learn", t0)
        else:
            t0 = self._start()
            if ret is None:
                ret, adv = self.advantages()
            b = self._bufs
            T = self.batch_size
            al, cl = update_step(self.actors, self.critic, self.optim_actor, self.optim_critic, b["feats"][:T],
                                 b["masks"][:T], b["actions"], ret, adv, self.gidx, self.midx, self.entropy_coef,
                                 self.max_grad_norm, self.group, self.dedup, self.grad_probe)
            self._mark("learn", t0)
        for a, x in zip(AGENTS, al):
            self.actor_loss_history[a].append(x)
        self.critic_loss_history.append(cl)
        self.repack()
        return al, cl

    def _update_gathered(self):
        """Experience gather into the learner (rank 0 of the group): the reference's
        transition_memory filled with every rank's transitions, finish_trajectory + _update
        over the whole batch (a2c.py:324-336), then the parameters broadcast back."""
        import time
        from . import distributed as D
        import torch.distributed as dist
        t0 = self._start()
        b = self._bufs
        T = self.batch_size
        slab = {"feats": b["feats"][:T], "masks": b["masks"][:T], "actions": b["actions"], "rewards": b["rewards"],
                "values": b["values"], "done": b["term"] | b["trunc"]}
        full = D.gather_slabs(slab, dst=0, group=self.group)
        t0 = self._mark("gather", t0)
        params = list(self.actors.parameters()) + list(self.critic.parameters())
        stats = torch.zeros(NA + 1, dtype=torch.float32, device=self.device)
        if dist.get_rank(self.group) == 0:
            cat = lambda x: x.movedim(0, -2).reshape(*x.shape[1:-1], -1)   # [W, ..., n] -> [..., W*n]  # noqa: E731
            g = {k: cat(v) for k, v in full.items()}
            del full
            ret, adv = self.gae_fn(g["rewards"], g["values"], g["done"], self.gamma, self.lamb, self.use_gae)
            al, cl = update_step(self.actors, self.critic, self.optim_actor, self.optim_critic, g["feats"], g["masks"],
                                 g["actions"], ret, adv, self.gidx, self.midx, self.entropy_coef,
                                 self.max_grad_norm, D.LOCAL, self.dedup, self.grad_probe)
            stats.copy_(torch.tensor(al + [cl], dtype=torch.float32))
        t0 = self._mark("learn", t0)
        D.broadcast_flat(params + [stats], src=0, group=self.group)
        self._mark("broadcast", t0)
        v = stats.cpu().tolist()
        return v[:NA], v[NA]

    @torch.no_grad()
    def batch_stats(self):
        """What the last collected batch looked like to the update (diagnostics, synchronising):
        per agent the share of samples whose action was forced (one valid action) and of 64-env
        tiles where every env was forced (k_policy skips those tiles' MLPs), and the number of
        distinct inputs each network saw (the grouped update runs each network once per
        distinct input)."""
        b = self._bufs
        T = self.batch_size
        m = b["masks"][:T].int()
        forced, tiles = {}, {}
        for i, a in enumerate(AGENTS):
            o, k = MASK_OFFS[i], N_ACTIONS[i]
            f = m[:, o:o + k, :].sum(1) == 1                     # [T, N]
            forced[a] = float(f.float().mean())
            n64 = (self.N // 64) * 64
            tiles[a] = float(f[:, :n64].reshape(T, -1, 64).all(-1).float().mean()) if n64 else 0.0
        g = RowGroups(group_keys(b["feats"][:T].contiguous()))
        return {"samples": T * self.N, "forced_share": forced, "forced_tile_share": tiles,
                "distinct_inputs": dict(zip(AGENTS, g.U[:NA])), "distinct_global_states": g.U[NA]}

    def exchange_bytes_per_batch(self):
        """Bytes one rank sends per batch: exchange="gather" the transition slab; "shard" the
        records the last batch sent to other ranks (measured: the combiner's output varies)."""
        if self.exchange == "shard":   # 0 before the first update has measured it
            return self.shard_info.get("bytes_sent_to_other_ranks", 0)
        T, N = self.batch_size, self.N
        per_env_step = GLOBAL_DIM * 4 + 29 + NA + NA * 8 + 4 + 1
        return T * N * per_env_step + N * 4

    def roll_over(self):
        """The last observation of the batch becomes the first of the next."""
        b = self._bufs
        b["feats"][0].copy_(b["feats"][self.batch_size])
        b["masks"][0].copy_(b["masks"][self.batch_size])

    def learn(self, total_timesteps, num_orders=25, seeds=None, deterministic=False, action_fn=None):
        """learn (a2c.py:254-388) on N envs: total_timesteps counts env-steps of this shard
        (N per vector step); an update every batch_size vector steps."""
        self.reset(seeds=seeds, num_orders=num_orders)
        steps = 0
        while steps < total_timesteps:
            self.collect(deterministic, action_fn)
            self.update()
            self.roll_over()
            steps += self.batch_size * self.N
        return self

    @torch.no_grad()
    def test(self, num_orders=5, max_steps=500, seeds=None, deterministic=True, trace=False, env=None,
             use_heuristic=False):
        """MultiAgentA2C.test (a2c.py:539-645) with the learned policy on every env: greedy
        actions (deterministic) until each env's episode ends or max_steps.  Returns per-env
        numpy arrays as the reference's test() dict (+ the actions [T, 8, N] with trace).
        Runs on `env` (a separate FJSPVecEnv, as the reference builds a fresh test env) or,
        by default, on the training env, which is reset afterwards with the training
        num_orders (the next collect() starts new episodes from fresh observations)."""
        on_train = env is None or env is self.env
        res = self._test(num_orders, max_steps, seeds, deterministic, trace, self.env if env is None else env,
                         use_heuristic)
        if on_train and self._bufs is not None:
            self.reset(num_orders=getattr(self, "num_orders", 25))
        return res

    @torch.no_grad()
    def _test(self, num_orders, max_steps, seeds, deterministic, trace, env, use_heuristic):
        import numpy as np
        from .vec_env import Buffers
        if use_heuristic:
            return env.evaluate("heuristic", num_orders=num_orders, max_steps=max_steps, seeds=seeds)
        N = env.num_envs
        env.reset(seeds=seeds, num_orders=num_orders)
        feats, masks = env.pack_a2c()
        b = Buffers(1, N, self.device, infos=True, feats=True)
        act = torch.zeros(NA, N, dtype=torch.uint8, device=self.device)
        val = torch.zeros(N, dtype=torch.float32, device=self.device)
        alive = torch.ones(N, dtype=torch.bool, device=self.device)
        steps = torch.zeros(N, dtype=torch.int64, device=self.device)
        by_agent = torch.zeros(NA, N, dtype=torch.float64, device=self.device)
        oc = torch.zeros(N, dtype=torch.int64, device=self.device)
        pk = torch.zeros(N, dtype=torch.int64, device=self.device)
        acts = []
        for t in range(int(max_steps)):
            if self.fused_policy:
                self.policy_fused(feats, masks, t, deterministic, act, val, gid0=env.env_id_base)
            else:
                act.copy_(self.policy(feats, masks, deterministic, t=t, gid0=env.env_id_base)[0])
            if trace:
                acts.append(act.cpu().numpy().copy())
            env.step(act, autoreset=False, buffers=b)
            by_agent += torch.where(alive, b.rewards[0], torch.zeros_like(by_agent))
            steps += alive.long()
            oc = torch.where(alive, b.orders_completed[0].long(), oc)
            pk = torch.where(alive, b.packaged[0].long(), pk)
            alive &= ~(b.term[0].bool() | b.trunc[0].bool())
            feats.copy_(b.feats[0])
            masks.copy_(b.masks[0])
            if not bool(alive.any()):
                break
        by_agent = by_agent.cpu().numpy()
        res = {"steps": steps.cpu().numpy(), "orders_completed": oc.cpu().numpy(),
               "products_packaged": pk.cpu().numpy(), "total_orders": num_orders,
               "rewards_by_agent": by_agent, "total_reward": np.cumsum(by_agent, axis=0)[-1]}
        if trace:
            res["actions"] = np.stack(acts) if acts else np.zeros((0, NA, N), np.uint8)
        return res

    # ------------------------------------------------------------ checkpoints (a2c.py:733-775)
    def state_dicts(self):
        return {
            "actor_nets": {a: self.actors.actor_state_dict(i) for i, a in enumerate(AGENTS)},
            "critic_net": {k: v.detach().cpu().clone() for k, v in self.critic.state_dict().items()},
            "obs_dims": dict(self.obs_dims),
            "act_dims": dict(self.act_dims),
            "global_obs_dim": GLOBAL_DIM,
            "possible_agents": list(AGENTS),
        }

    def save_model(self, path):
        import os
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        torch.save(self.state_dicts(), path)

    def load_model(self, path):
        """Loads a reference checkpoint (or one written by save_model) without executing
        anything from the file (load_checkpoint: weights_only=True)."""
        self.load_state_dicts(load_checkpoint(path))

    def load_state_dicts(self, ck):
        """load_model (a2c.py:756-775): only the agents the checkpoint holds are overwritten
        (the others keep their weights); the critic if present."""
        nets = []
        for i, a in enumerate(AGENTS):
            net = ActorNet(OBS_DIMS[i], N_ACTIONS[i], self.actors.hidden)
            sd = ck.get("actor_nets", {}).get(a)
            if sd is None:
                sd = self.actors.actor_state_dict(i)
            net.load_state_dict(sd)
            nets.append(net)
        self.actors.load_actor_nets([n.to(self.device) for n in nets])
        if ck.get("critic_net") is not None:
            self.critic.load_state_dict(ck["critic_net"])
        if getattr(self, "fused_policy", False):
            self.repack()


def _checkpoint_globals():
    """The only non-tensor globals a reference checkpoint pickles: a2c.py:80 stores
    act_space.n — a numpy int64 scalar under gymnasium — into act_dims, which save_model
    (a2c.py:745-753) pickles as numpy.core.multiarray.scalar(dtype('int64'), bytes).  Under
    numpy 2 the function lives in numpy._core, so it is allowlisted under its pickled name."""
    import numpy as np
    try:
        from numpy._core import multiarray as ma
    except ImportError:                                   # numpy 1.x
        from numpy.core import multiarray as ma
    return [(ma.scalar, "numpy.core.multiarray.scalar"), np.dtype, type(np.dtype(np.int64))]


def load_checkpoint(path):
    """A reference (a2c.py:733-775) or save_model checkpoint as a dict, read with
    torch.load(weights_only=True) and an allowlist of exactly the numpy scalar global and the
    int64 dtype class (nothing from the file is executed; there is no weights_only=False
    fallback).  obs_dims / act_dims / global_obs_dim come back as Python ints."""
    with torch.serialization.safe_globals(_checkpoint_globals()):
        ck = torch.load(path, map_location="cpu", weights_only=True)
    for k in ("obs_dims", "act_dims"):
        if isinstance(ck.get(k), dict):
            ck[k] = {a: int(v) for a, v in ck[k].items()}
    if "global_obs_dim" in ck:
        ck["global_obs_dim"] = int(ck["global_obs_dim"])
    return ck


def load_npz_weights(path):
    """A checkpoint's tensors stored as an .npz (w_actor.<agent>.<param>, w_critic.<param>;
    tests/golden/gen_trained_golden.py) -> the load_state_dicts dict."""
    import numpy as np
    z = np.load(path)
    ck = {"actor_nets": {}, "critic_net": {}}
    for k in z.files:
        if k.startswith("w_actor."):
            _, a, p = k.split(".", 2)
            ck["actor_nets"].setdefault(a, {})[p] = torch.from_numpy(z[k].copy())
        elif k.startswith("w_critic."):
            ck["critic_net"][k[len("w_critic."):]] = torch.from_numpy(z[k].copy())
    return ck


def num_params(model):
    return sum(math.prod(p.shape) for p in model.parameters())
