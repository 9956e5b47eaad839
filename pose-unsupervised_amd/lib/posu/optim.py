"""Adam on the HIP kernel (posu_adam_step, include/posu.h): a drop-in for the reference's
optimizer, torch.optim.Adam (utils/utils.py:79-83, stepped by core/function.py:366), for f32
parameters on the GPU.

Same hyper-parameters, state layout ('step', 'exp_avg', 'exp_avg_sq' per parameter, so
state_dict / load_state_dict and a switch to or from torch.optim.Adam keep working) and update
rule; the arithmetic is f32 and agrees with torch's kernels within rounding, not bit for bit.
Every parameter of a group with the same step count goes to one call (a few launches for the
whole network).  amsgrad / maximize / complex parameters are refused.
"""
import ctypes

import numpy as np
import torch

from . import _native as nat

_REC = np.dtype([('p', '<u8'), ('g', '<u8'), ('m', '<u8'), ('v', '<u8'), ('n', '<i8')])
assert _REC.itemsize == 40   # sizeof(posu_adam_tensor)


class Adam(torch.optim.Adam):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            if group.get('amsgrad') or group.get('maximize') or group.get('differentiable'):
                raise NotImplementedError('posu.optim.Adam: amsgrad / maximize / differentiable are not supported')
            # every parameter is checked before any state changes: a refusal leaves the optimizer as it was
            params = [p for p in group['params'] if p.grad is not None]
            for p in params:
                if p.grad.is_sparse or p.is_complex() or p.dtype != torch.float32:
                    raise NotImplementedError('posu.optim.Adam: dense f32 parameters only')
                nat.require_cuda(p, p.grad)
                st = self.state[p]
                if not p.is_contiguous() or (len(st) and not (st['exp_avg'].is_contiguous() and
                                                              st['exp_avg_sq'].is_contiguous())):
                    raise NotImplementedError('posu.optim.Adam: contiguous parameters and state only')
            by_step = {}
            for p in params:
                st = self.state[p]
                if len(st) == 0:   # torch.optim.Adam's state (step on the host, as its non-fused form)
                    st['step'] = torch.tensor(0.0)
                    st['exp_avg'] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st['step'] += 1
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                by_step.setdefault((int(st['step'].item()), p.device), []).append((p, g, st))
            beta1, beta2 = group['betas']
            for (step, dev), items in by_step.items():
                rec = np.zeros(len(items), dtype=_REC)
                for i, (p, g, st) in enumerate(items):
                    rec[i] = (p.data_ptr(), g.data_ptr(), st['exp_avg'].data_ptr(), st['exp_avg_sq'].data_ptr(),
                              p.numel())
                with torch.cuda.device(dev):
                    nat.call('posu_adam_step', rec.ctypes.data_as(ctypes.c_void_p), len(items), float(group['lr']),
                             float(beta1), float(beta2), float(group['eps']), float(group['weight_decay']), step,
                             nat.stream_of(dev))
        return loss
