"""Fused RAdam for the discriminator of the train_stft step.

``FusedRAdam`` is radam.py's rectified Adam (radam.py:35-99, the optimizer
``RAdam(net_d.parameters(), 1e-4)`` of train_stft.py:97) as one HIP launch
over every parameter tensor (``vits_radam_step``, csrc/optim.hip).  It
implements GradScaler's optimizer contract (``_step_supports_amp_scaling``:
the scaler hands over ``found_inf`` / ``grad_scale`` device tensors instead
of syncing the host on ``found_inf.item()``), so the D step of the train
loop is sync-free and graph-capturable.  The step count and the
rectification scalars (N_sma, step size) live on the device; one count per
param group, which every parameter of the group shares (radam.py keeps one
per parameter, all equal since they are stepped together).

State layout per parameter: ``exp_avg``, ``exp_avg_sq`` (fp32, like
radam.py) and ``step`` (a view of the group's device counter).  A loaded
state (``load_state_dict``: this optimizer's own state_dict or a reference
``D_*.pth`` whose per-parameter ``step`` is a Python int) seeds the group
counter, so a resumed run continues at t+1 instead of re-running RAdam's
warm-up on already-warm moments.

The learning rate may be a float or a device tensor (``lr=torch.tensor(..)``):
a tensor is read by the kernel at run time, so an lr scheduler's in-place
update (torch's schedulers ``fill_`` tensor lrs) reaches a graph-captured
step.  ROCm tensors only; ``RAdam`` below is radam.py's update in plain
torch for CPU tensors (the CPU unit tests of the train loop).
"""
from __future__ import annotations

import math

import torch

from . import _lib
from ._lib import RadamTensor, check


class FusedRAdam(torch.optim.Optimizer):
    _step_supports_amp_scaling = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0):
        if float(lr) < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid RAdam hyper-parameters")
        if isinstance(lr, torch.Tensor) and (lr.numel() != 1 or lr.device.type != "cuda"):
            raise ValueError("a tensor lr must be a one-element ROCm tensor")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps,
                                      weight_decay=weight_decay))
        self._scal = {}

    def _group_scal(self, gi: int, device) -> torch.Tensor:
        s = self._scal.get(gi)
        if s is None:
            s = torch.zeros(8, dtype=torch.float32, device=device)
            self._scal[gi] = s
        return s

    def state_dict(self):
        """torch's state_dict with radam.py's types: each ``step`` a Python
        int (radam.py:69 counts with ``+= 1``), a tensor ``lr`` as a float,
        so a ``D_*.pth`` written here loads into the reference's RAdam."""
        sd = super().state_dict()
        # torch hands out the live per-parameter state dicts: copy them before
        # rewriting ``step``, or the live entry (a view of the group's device
        # counter) would be replaced by a frozen int
        sd["state"] = {k: dict(v) for k, v in sd["state"].items()}
        for st in sd["state"].values():
            if isinstance(st.get("step"), torch.Tensor):
                st["step"] = int(round(float(st["step"])))
        sd["param_groups"] = [dict(g) for g in sd["param_groups"]]
        for g in sd["param_groups"]:
            for k in ("lr", "initial_lr"):
                if isinstance(g.get(k), torch.Tensor):
                    g[k] = float(g[k])
        return sd

    def load_state_dict(self, state_dict):
        """torch's load, then seed each group's device step counter from the
        loaded per-parameter ``step`` (tensor or int, all equal within a
        group as radam.py steps them together) and re-point every state's
        ``step`` at the counter view.  The counter and the moments are
        written IN PLACE when they already exist (a captured step keeps
        pointing at them), and a tensor ``lr`` keeps its object
        (the loaded value is copied into it)."""
        old = {p: dict(self.state[p]) for p in self.state}
        old_lr = [(g.get("lr"), g.get("initial_lr")) for g in self.param_groups]
        super().load_state_dict(state_dict)
        for gi, group in enumerate(self.param_groups):
            for k, prev in zip(("lr", "initial_lr"), old_lr[gi]):
                if isinstance(prev, torch.Tensor) and k in group and group[k] is not prev:
                    prev.fill_(float(group[k]))
                    group[k] = prev
            steps = [self.state[p]["step"] for p in group["params"]
                     if p in self.state and "step" in self.state[p]]
            if not steps:
                continue
            t = max(float(s) for s in steps)
            dev = group["params"][0].device
            scal = self._group_scal(gi, dev)
            scal[0] = t
            for p in group["params"]:
                st = self.state.get(p)
                if st and "step" in st:
                    st["step"] = scal[0:1]
                    for k in ("exp_avg", "exp_avg_sq"):
                        if k in st:
                            new = st[k].to(device=p.device, dtype=torch.float32).contiguous()
                            prev = old.get(p, {}).get(k)
                            if isinstance(prev, torch.Tensor) and prev.shape == new.shape:
                                prev.copy_(new)
                                new = prev
                            st[k] = new

    @staticmethod
    def _lr_args(group, dev):
        lr = group["lr"]
        if isinstance(lr, torch.Tensor):
            if lr.dtype != torch.float64 or lr.device != dev:
                # the kernel reads a device double; keep the group's tensor
                # (the one a scheduler updates) as that double
                lr = lr.to(device=dev, dtype=torch.float64)
                group["lr"] = lr
            return 0.0, lr.data_ptr()
        return float(lr), None

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        found_inf = getattr(self, "found_inf", None)
        grad_scale = getattr(self, "grad_scale", None)
        lib = _lib.load()
        for gi, group in enumerate(self.param_groups):
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            dev = ps[0].device
            if dev.type != "cuda":
                raise _lib.VitsAmdError("FusedRAdam needs ROCm tensors; there is no CPU path")
            scal = self._group_scal(gi, dev)
            arr = (RadamTensor * len(ps))()
            for i, p in enumerate(ps):
                if p.dtype != torch.float32 or not p.is_contiguous() or \
                        p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                    raise _lib.VitsAmdError("FusedRAdam: fp32 contiguous params / grads only")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = scal[0:1]
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                arr[i].param = p.data_ptr()
                arr[i].grad = p.grad.data_ptr()
                arr[i].exp_avg = st["exp_avg"].data_ptr()
                arr[i].exp_avg_sq = st["exp_avg_sq"].data_ptr()
                arr[i].numel = p.numel()
            fi = None
            if found_inf is not None:
                fi = found_inf.to(device=dev, dtype=torch.float32)
            gs = None
            if grad_scale is not None:
                gs = grad_scale.to(device=dev, dtype=torch.float32)
            b1, b2 = group["betas"]
            lr, lr_ptr = self._lr_args(group, dev)
            check(lib.vits_radam_step(arr, len(ps), scal.data_ptr(),
                                      None if fi is None else fi.data_ptr(),
                                      None if gs is None else gs.data_ptr(),
                                      lr, lr_ptr, float(b1), float(b2), float(group["eps"]),
                                      float(group["weight_decay"]),
                                      torch.cuda.current_stream(dev).cuda_stream),
                  "vits_radam_step")
        return loss


class RAdam(torch.optim.Optimizer):
    """radam.py's rectified Adam (radam.py:35-99) in plain torch, for CPU
    tensors: per-parameter int step, rectification when N_sma >= 5 (torch's
    own RAdam uses > 5), weight decay applied to the parameter before the
    update (radam.py:87-88; not an L2 term on the gradient).  Scalars in
    Python doubles as the reference computes them."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid RAdam hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps,
                                      weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            b1, b2 = group["betas"]
            lr = float(group["lr"])
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad.float()
                w = p.float()
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(w)
                    st["exp_avg_sq"] = torch.zeros_like(w)
                m, v = st["exp_avg"], st["exp_avg_sq"]
                v.mul_(b2).addcmul_(g, g, value=1 - b2)
                m.mul_(b1).add_(g, alpha=1 - b1)
                st["step"] = t = int(st["step"]) + 1
                b2t = b2 ** t
                nmax = 2.0 / (1.0 - b2) - 1.0
                n = nmax - 2.0 * t * b2t / (1.0 - b2t)
                if n >= 5:
                    s = math.sqrt((1 - b2t) * (n - 4) / (nmax - 4) * (n - 2) / n * nmax
                                  / (nmax - 2)) / (1 - b1 ** t)
                else:
                    s = 1.0 / (1 - b1 ** t)
                if group["weight_decay"] != 0:
                    w.add_(w, alpha=-group["weight_decay"] * lr)
                if n >= 5:
                    w.addcdiv_(m, v.sqrt().add_(group["eps"]), value=-s * lr)
                else:
                    w.add_(m, alpha=-s * lr)
                p.copy_(w)
        return loss
