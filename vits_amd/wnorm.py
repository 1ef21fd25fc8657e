"""Weight / spectral normalisation of a whole network in a few HIP launches
(csrc/wnorm.hip, C-ABI ``vits_weight_norm_*`` / ``vits_spectral_norm_*``).

The reference recomputes every reparametrised weight in a per-layer forward
pre-hook: legacy ``torch.nn.utils.weight_norm`` on the generator
(modules.py:58-109, models.py:233; ~216 layers) and
``torch.nn.utils.spectral_norm`` on the MWSD discriminators (mrd.py; 85
layers, one power iteration per training forward).  In the train_stft step
that is ~2,500 small kernels per iteration.  Here:

* ``WeightNormCache(net_g).active()`` computes every weight-normed layer's
  effective weight in ONE launch (``_WeightNormAll``) and serves it to the
  layers' forwards (``ops.weight_norm_effective``); their gradients flow
  back into one backward launch for all ``weight_g`` / ``weight_v``.
* ``spectral_norm_all`` runs the power iteration, sigma and W / sigma of
  every layer in one launch and the backward of W / sigma(W) in another;
  ``discriminators.GroupedSpectralNorm`` uses it on the GPU.

Same parameters, buffers (``weight_u`` / ``weight_v`` updated in place) and
formulas as the torch hooks (float32; the spectral norm reproduces the fp16
rounding of the reference's autocast ``mv`` when called inside fp16
autocast).  GPU only: these are product paths without a CPU fallback; the
callers keep torch's hooks on CPU.
"""
from __future__ import annotations

import contextlib

import torch
from torch.nn.utils.spectral_norm import SpectralNorm
from torch.nn.utils.weight_norm import WeightNorm

from . import _lib, ops
from ._lib import SnormLayer, WnormLayer, check

FUSED_NORMS = True  # test switch (both norms)
FUSED_WN = FUSED_SN = True  # per-kind switches (diagnostics)


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


# ---------------------------------------------------------------------------
# weight norm
# ---------------------------------------------------------------------------


class _WeightNormAll(torch.autograd.Function):
    """(g_0..g_{n-1}, v_0..v_{n-1}) -> (w_0..w_{n-1}), w = v * (g / ||v_row||)."""

    @staticmethod
    def forward(ctx, n: int, *gv):
        gs, vs = gv[:n], gv[n:]
        ws = [torch.empty_like(v) for v in vs]
        rows = sum(v.shape[0] for v in vs)
        norms = torch.empty(rows, device=vs[0].device, dtype=torch.float32)
        arr = (WnormLayer * n)()
        for i, (g, v, w) in enumerate(zip(gs, vs, ws)):
            arr[i].v, arr[i].g, arr[i].w = v.data_ptr(), g.data_ptr(), w.data_ptr()
            arr[i].rows, arr[i].cols = v.shape[0], v.numel() // v.shape[0]
        check(_lib.load().vits_weight_norm_forward(arr, n, norms.data_ptr(), _stream(norms)),
              "vits_weight_norm_forward")
        ctx.n = n
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(*gs, *vs, norms)
        return tuple(ws)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, *dws):
        n = ctx.n
        saved = ctx.saved_tensors
        gs, vs, norms = saved[:n], saved[n:2 * n], saved[2 * n]
        dgs, dvs = [None] * n, [None] * n
        lib = _lib.load()
        # runs of layers with a gradient (the norms of a launch are consecutive)
        row0, i = 0, 0
        while i < n:
            if dws[i] is None:
                row0 += vs[i].shape[0]
                i += 1
                continue
            j = i
            while j < n and dws[j] is not None:
                j += 1
            arr = (WnormLayer * (j - i))()
            keep = []
            for a, q in enumerate(range(i, j)):
                dw = dws[q].contiguous()
                keep.append(dw)
                dgs[q], dvs[q] = torch.empty_like(gs[q]), torch.empty_like(vs[q])
                e = arr[a]
                e.v, e.g, e.dw = vs[q].data_ptr(), gs[q].data_ptr(), dw.data_ptr()
                e.dv, e.dg = dvs[q].data_ptr(), dgs[q].data_ptr()
                e.rows, e.cols = vs[q].shape[0], vs[q].numel() // vs[q].shape[0]
            check(lib.vits_weight_norm_backward(arr, j - i, norms.data_ptr() + 4 * row0,
                                                _stream(norms)), "vits_weight_norm_backward")
            row0 += sum(vs[q].shape[0] for q in range(i, j))
            i = j
        return (None, *dgs, *dvs)


def _weight_norm_hook(m: torch.nn.Module):
    for h in m._forward_pre_hooks.values():
        if isinstance(h, WeightNorm):
            return h
    return None


class WeightNormCache:
    """Every legacy weight-normed (dim 0, fp32) layer of ``root``: while
    ``active()``, ``ops.weight_norm_effective(layer)`` returns the weight
    computed for all of them by one ``vits_weight_norm_forward`` launch."""

    def __init__(self, root: torch.nn.Module, groups=("",)):
        """groups: one tuple of module-name prefixes per group (a plain
        string is a one-prefix group; a module joins the first group with a
        matching prefix); each group's weights come from one launch and go
        back in one (its backward runs as soon as that group's last weight
        gradient is in: the decoder's long before the text encoder's, so its
        gradients can be all-reduced while the rest of the backward runs -
        train._GradBuckets)."""
        groups = [(g,) if isinstance(g, str) else tuple(g) for g in groups]
        self.mods = []
        self.groups = [[] for _ in groups]
        for name, m in root.named_modules():
            h = _weight_norm_hook(m)
            if h is None or h.dim != 0:
                continue
            g, v = getattr(m, h.name + "_g"), getattr(m, h.name + "_v")
            if g.dtype == v.dtype == torch.float32 and v.is_cuda and v.is_contiguous() \
                    and g.is_contiguous() and g.numel() == v.shape[0]:
                self.mods.append((m, h.name))
                gi = next(i for i, pres in enumerate(groups)
                          if any((name + ".").startswith(pre) for pre in pres))
                self.groups[gi].append((m, h.name))
        self.groups = [grp for grp in self.groups if grp]

    def weights(self):
        out = {}
        for grp in self.groups:
            gs = [getattr(m, n + "_g") for m, n in grp]
            vs = [getattr(m, n + "_v") for m, n in grp]
            ws = _WeightNormAll.apply(len(grp), *gs, *vs)
            out.update({m: w for (m, _), w in zip(grp, ws)})
        return out

    @contextlib.contextmanager
    def active(self):
        if not (FUSED_NORMS and FUSED_WN and self.mods):
            yield
            return
        prev = ops.set_weight_cache(self.weights())
        try:
            yield
        finally:
            ops.set_weight_cache(prev)


# ---------------------------------------------------------------------------
# spectral norm
# ---------------------------------------------------------------------------


def _sn_forward(layers, training: bool, emu16: bool, Ws):
    """One launch: (outs, saved, offs, shapes) of W / sigma(W) for every W
    (power iteration on the layers' u / v buffers when training)."""
    n = len(Ws)
    # layers: (u, v, eps, cl) - cl = C > 0: W / sigma as the fp16
    # channels-last image the autocast MIOpen conv would cast it to
    outs = [torch.empty(W.shape, device=W.device, dtype=torch.float16,
                        memory_format=torch.channels_last) if lay[3] else torch.empty_like(W)
            for W, lay in zip(Ws, layers)]
    shapes = [(W.shape[0], W.numel() // W.shape[0]) for W in Ws]
    offs, tot = [], 0
    for r, c in shapes:
        offs.append(tot)
        tot += 1 + r + c
    saved = torch.empty(tot, device=Ws[0].device, dtype=torch.float32)
    arr = (SnormLayer * n)()
    for i, (W, (u, v, eps, cl)) in enumerate(zip(Ws, layers)):
        e = arr[i]
        e.w, e.u, e.v, e.w_sn = W.data_ptr(), u.data_ptr(), v.data_ptr(), outs[i].data_ptr()
        e.saved = saved.data_ptr() + 4 * offs[i]
        e.rows, e.cols = shapes[i]
        e.eps = eps
        e.cl_channels = cl
    check(_lib.load().vits_spectral_norm_forward(arr, n, int(training), int(emu16),
                                                 _stream(saved)), "vits_spectral_norm_forward")
    return outs, saved, offs, shapes


def _sn_backward(Ws, saved, offs, shapes, emu16, cls, gs, need):
    """dW of W / sigma(W) for the layers with a gradient (one launch)."""
    n = len(Ws)
    dWs = [None] * n
    idx = [i for i in range(n) if gs[i] is not None and need[i]]
    if idx:
        arr = (SnormLayer * len(idx))()
        keep = []
        for a, i in enumerate(idx):
            if cls[i]:
                g = gs[i].to(torch.float16).contiguous(memory_format=torch.channels_last)
            else:
                g = gs[i].float().contiguous()
            keep.append(g)
            dWs[i] = torch.empty_like(Ws[i])
            e = arr[a]
            e.w, e.dw_sn, e.dw = Ws[i].data_ptr(), g.data_ptr(), dWs[i].data_ptr()
            e.saved = saved.data_ptr() + 4 * offs[i]
            e.rows, e.cols = shapes[i]
            e.cl_channels = cls[i]
        lib = _lib.load()
        nws = lib.vits_spectral_norm_workspace(arr, len(idx))
        ws = torch.empty(max(1, nws), device=saved.device, dtype=torch.float32)
        check(lib.vits_spectral_norm_backward(arr, len(idx), int(emu16), ws.data_ptr(),
                                              ws.numel(), _stream(saved)),
              "vits_spectral_norm_backward")
    return dWs


class _SpectralNormAll(torch.autograd.Function):
    """(W_0..W_{n-1}) -> (W_0 / sigma_0, ...); power iteration on the u / v
    buffers of ``layers`` (a list of (u, v, eps, cl)) in training mode."""

    @staticmethod
    def forward(ctx, layers, training: bool, emu16: bool, *Ws):
        outs, saved, offs, shapes = _sn_forward(layers, training, emu16, Ws)
        ctx.offs, ctx.shapes, ctx.emu16 = offs, shapes, emu16
        ctx.cls = [lay[3] for lay in layers]
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(*Ws, saved)
        return tuple(outs)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, *gs):
        saved_t = ctx.saved_tensors
        Ws, saved = saved_t[:-1], saved_t[-1]
        dWs = _sn_backward(Ws, saved, ctx.offs, ctx.shapes, ctx.emu16, ctx.cls, gs,
                           ctx.needs_input_grad[3:])
        return (None, None, None, *dWs)


class _SpectralNormAll2(torch.autograd.Function):
    """Two consecutive training-mode spectral norms of the same weights (the
    D(real) and D(fake) forwards of train_stft.py:198-200, one power
    iteration each) as ONE autograd node: (W_0..W_{n-1}) -> (W_i / sigma1_i
    for every i, then W_i / sigma2_i for every i).  Its backward runs one
    backward launch per pass and sums them with one multi-tensor add, where
    two nodes would make autograd add each layer's two gradients one by one."""

    @staticmethod
    def forward(ctx, layers, emu16: bool, *Ws):
        outs1, saved1, offs, shapes = _sn_forward(layers, True, emu16, Ws)
        outs2, saved2, _, _ = _sn_forward(layers, True, emu16, Ws)
        ctx.offs, ctx.shapes, ctx.emu16 = offs, shapes, emu16
        ctx.cls = [lay[3] for lay in layers]
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(*Ws, saved1, saved2)
        return tuple(outs1) + tuple(outs2)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, *gs):
        n = len(gs) // 2
        saved_t = ctx.saved_tensors
        Ws, saved1, saved2 = saved_t[:n], saved_t[n], saved_t[n + 1]
        need = ctx.needs_input_grad[2:]
        d1 = _sn_backward(Ws, saved1, ctx.offs, ctx.shapes, ctx.emu16, ctx.cls, gs[:n], need)
        d2 = _sn_backward(Ws, saved2, ctx.offs, ctx.shapes, ctx.emu16, ctx.cls, gs[n:], need)
        both = [i for i in range(n) if d1[i] is not None and d2[i] is not None]
        if both:
            torch._foreach_add_([d1[i] for i in both], [d2[i] for i in both])
        return (None, None, *[d1[i] if d1[i] is not None else d2[i] for i in range(n)])


def spectral_norm_supported(W: torch.Tensor) -> bool:
    if not (W.is_cuda and W.dtype == torch.float32 and W.is_contiguous() and W.dim() >= 2):
        return False
    return bool(_lib.load().vits_spectral_norm_supported(W.shape[0], W.numel() // W.shape[0]))


def spectral_norm_all2(Ws, layers, cl16=None):
    """spectral_norm_all twice in training mode (two power iterations, the
    u / v buffers updated by each) as one autograd node: (the first pass's
    W / sigma list, the second pass's)."""
    dev = Ws[0].device.type
    emu16 = torch.is_autocast_enabled(dev) and torch.get_autocast_dtype(dev) == torch.float16
    cl16 = cl16 or [False] * len(Ws)
    lay = [(u, v, eps, W.shape[1] if (emu16 and c and W.dim() == 4) else 0)
           for W, (u, v, eps), c in zip(Ws, layers, cl16)]
    outs = _SpectralNormAll2.apply(lay, bool(emu16), *Ws)
    return list(outs[:len(Ws)]), list(outs[len(Ws):])


def spectral_norm_all(Ws, layers, training: bool, cl16=None):
    """W / sigma for every weight (torch.nn.utils.spectral_norm semantics, dim
    0, one power iteration when training); ``layers``: (u, v, eps) per W.
    Inside an fp16 autocast region the reference's fp16 ``mv`` rounding is
    reproduced, and the 4-D weights flagged in ``cl16`` come out as the fp16
    channels-last tensors the autocast MIOpen convs consume (the cast and
    layout copy those convs would make, done in the same kernel)."""
    dev = Ws[0].device.type
    emu16 = torch.is_autocast_enabled(dev) and torch.get_autocast_dtype(dev) == torch.float16
    cl16 = cl16 or [False] * len(Ws)
    lay = [(u, v, eps, W.shape[1] if (emu16 and c and W.dim() == 4) else 0)
           for W, (u, v, eps), c in zip(Ws, layers, cl16)]
    return _SpectralNormAll.apply(lay, bool(training), bool(emu16), *Ws)


def spectral_norm_hook(m: torch.nn.Module, name: str):
    for h in m._forward_pre_hooks.values():
        if isinstance(h, SpectralNorm) and h.name == name:
            return h
    return None


__all__ = ["WeightNormCache", "spectral_norm_all", "spectral_norm_all2", "spectral_norm_supported",
           "FUSED_NORMS"]
