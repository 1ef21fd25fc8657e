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
radam.py) and ``step`` (a view of the group's device counter).
ROCm tensors only: the CPU unit tests of the train loop use
``torch.optim.RAdam`` (same update; vits_amd.train picks it off-GPU).
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import RadamTensor, check


class FusedRAdam(torch.optim.Optimizer):
    _step_supports_amp_scaling = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid RAdam hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps,
                                      weight_decay=weight_decay))
        self._scal = {}

    def _group_scal(self, gi: int, device) -> torch.Tensor:
        s = self._scal.get(gi)
        if s is None:
            s = torch.zeros(8, dtype=torch.float32, device=device)
            self._scal[gi] = s
        return s

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
            check(lib.vits_radam_step(arr, len(ps), scal.data_ptr(),
                                      None if fi is None else fi.data_ptr(),
                                      None if gs is None else gs.data_ptr(),
                                      float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                                      float(group["weight_decay"]),
                                      torch.cuda.current_stream(dev).cuda_stream),
                  "vits_radam_step")
        return loss
