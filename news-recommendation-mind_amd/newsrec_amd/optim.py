"""Adam on the HIP ``nr_adam`` kernel — a drop-in for the ``torch.optim.Adam`` that
utils/Manager.py:404-413 builds (two param groups, default betas/eps, no weight decay)."""
import torch

from . import kernels as K


class FusedAdam(torch.optim.Optimizer):
    """``capturable=True`` keeps each parameter's step count on the device (one multi-tensor
    add per step, bias corrections formed in the kernel), so ``step()`` can be captured in a
    graph and replayed — torch.optim.Adam(capturable=True) semantics."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, capturable=False):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.capturable = capturable

    @torch.no_grad()
    def step(self, closure=None, grad_scale=1.0):
        """``grad_scale`` multiplies every gradient as it is read (the data-parallel 1/world
        mean of GradSync), saving a separate scaling pass over the gradients."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        todo = []
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = (torch.zeros((), dtype=torch.int64, device=p.device) if self.capturable else 0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                todo.append((group, p, st))
        if self.capturable:
            steps = [st["step"] for _, _, st in todo]
            if steps:
                torch._foreach_add_(steps, 1)
        # one nr_adam_multi call per (betas, eps, weight_decay) combination: every tensor of the
        # step in a few launches instead of one launch per parameter
        batches = {}
        for group, p, st in todo:
            if not self.capturable:
                st["step"] += 1
            g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
            key = (tuple(group["betas"]), group["eps"], group["weight_decay"])
            batches.setdefault(key, []).append((p, g, st["exp_avg"], st["exp_avg_sq"], group["lr"], st["step"]))
        for (betas, eps, wd), entries in batches.items():
            K.adam_multi(entries, betas[0], betas[1], eps, wd, grad_scale)
        return loss
