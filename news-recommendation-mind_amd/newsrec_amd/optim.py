"""Adam on the HIP ``nr_adam`` kernel — a drop-in for the ``torch.optim.Adam`` that
utils/Manager.py:404-413 builds (two param groups, default betas/eps, no weight decay)."""
import weakref

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
        # capturable: each group's lr lives on the device too (read by the kernel), so a graph
        # replay follows group["lr"] changes (a warmup scheduler, Manager.py:415-420) once
        # sync_lr() has copied them over -- step() does it when not capturing, GraphedStep before
        # every replay
        self._lr_dev, self._lr_host = {}, {}

    def sync_lr(self):
        """Copy every group's host lr into its device scalar (only the ones that changed)."""
        for i, group in enumerate(self.param_groups):
            t = self._lr_dev.get(i)
            if t is None:
                dev = next((p.device for p in group["params"]), None)
                if dev is None:
                    continue
                t = self._lr_dev[i] = torch.empty((), dtype=torch.float32, device=dev)
                self._lr_host[i] = None
            if self._lr_host[i] != group["lr"]:
                t.fill_(float(group["lr"]))
                self._lr_host[i] = group["lr"]

    @torch.no_grad()
    def step(self, closure=None, grad_scale=1.0):
        """``grad_scale`` multiplies every gradient as it is read (the data-parallel 1/world
        mean of GradSync), saving a separate scaling pass over the gradients."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        todo = []
        if self.capturable and not torch.cuda.is_current_stream_capturing():
            self.sync_lr()
        for gi, group in enumerate(self.param_groups):
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                # a table sharded across ranks (dist.GradSync(shard_tables=True)): this rank updates
                # rows [row0, row0 + rows) only, with moments for those rows
                shard = getattr(p, "_nr_shard", None)
                if shard is not None and shard[1] == 0:
                    continue
                if len(st) == 0:
                    st["step"] = (torch.zeros((), dtype=torch.int64, device=p.device) if self.capturable else 0)
                    like = p if shard is None else p[shard[0]:shard[0] + shard[1]]
                    st["exp_avg"] = torch.zeros_like(like, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(like, memory_format=torch.contiguous_format)
                todo.append((gi, group, p, st))
        # capturable: the device step counts are advanced by the Adam launch itself
        # (nr_adam_multi_step: the bias corrections use count + 1, the last workgroup adds 1)
        # one nr_adam_multi call per (betas, eps, weight_decay) combination: every tensor of the
        # step in a few launches instead of one launch per parameter
        batches = {}
        for gi, group, p, st in todo:
            if not self.capturable:
                st["step"] += 1
            g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
            key = (tuple(group["betas"]), group["eps"], group["weight_decay"])
            lr = self._lr_dev[gi] if self.capturable else group["lr"]
            shard = getattr(p, "_nr_shard", None)
            if shard is not None:
                r0, n = shard
                batches.setdefault(key, []).append((p.data[r0:r0 + n], g[r0:r0 + n], st["exp_avg"], st["exp_avg_sq"],
                                                    lr, st["step"]))
                continue
            ent = (p, g, st["exp_avg"], st["exp_avg_sq"], lr, st["step"])
            # a row-sparse table gradient (functions.LOCAL_ROW_GRAD) carries per-row "touched" flags:
            # the kernel skips reading the rows known to be zero
            # rt = (that buffer, or a weak reference to the .grad tensor they were bound to, flags, its
            # version counter): the flags hold only while p.grad is that tensor, unmodified since
            # (functions._LocalRowGrad, functions._word_row_flags)
            rt = getattr(p, "_nr_row_touched", None)
            if rt is not None:
                if isinstance(rt[0], weakref.ref):
                    ok = rt[0]() is p.grad
                else:
                    ok = p.grad.data_ptr() == rt[0].data_ptr()
                if ok and p.grad._version == rt[2]:
                    ent = ent + (rt[1],)
            batches.setdefault(key, []).append(ent)
        for (betas, eps, wd), entries in batches.items():
            K.adam_multi(entries, betas[0], betas[1], eps, wd, grad_scale, advance_steps=self.capturable)
        return loss
