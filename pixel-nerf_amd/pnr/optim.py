"""Adam for the training step: torch.optim.Adam (the reference's optimizer, train.py / trainlib)
whose update of HIP fp32 parameters is ONE ``pnr_adam_step`` launch over every parameter of the
step (csrc/optim.hip), instead of torch's multi-tensor launches.

Same constructor, hyper-parameters, ``state`` (``step`` as a CPU tensor, ``exp_avg``,
``exp_avg_sq``) and ``state_dict`` as ``torch.optim.Adam``, so checkpoints move between the two.
Configurations the kernel does not implement (amsgrad, maximize, capturable, differentiable,
fused, a tensor lr, CPU / non-fp32 / sparse / non-contiguous tensors) step through torch's own
implementation of the reference's algorithm.
"""
import numpy as np
import torch

__all__ = ["Adam"]

CHUNK = 8192   # elements per workgroup (a multiple of 4: chunk starts stay 16-B aligned)


class Adam(torch.optim.Adam):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, **kw):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad, **kw)
        self._pinned = None      # host staging of the chunk table
        self._table = None       # device chunk table
        self._copied = None      # event after the last table upload

    @staticmethod
    def _group_ok(group):
        return not (group["amsgrad"] or group.get("maximize") or group.get("capturable")
                    or group.get("differentiable") or group.get("fused") or torch.is_tensor(group["lr"]))

    @staticmethod
    def _tensor_ok(p):
        g = p.grad
        return (p.is_cuda and p.dtype == torch.float32 and not g.is_sparse and g.dtype == torch.float32
                and p.is_contiguous() and g.is_contiguous() and g.device == p.device)

    @torch.no_grad()
    def step(self, closure=None):
        live = [(grp, [p for p in grp["params"] if p.grad is not None]) for grp in self.param_groups]
        if not all(self._group_ok(grp) and all(self._tensor_ok(p) for p in ps) for grp, ps in live):
            return super().step(closure)
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for grp, ps in live:
            # one launch per (device, step count): the parameters of a step normally share both
            runs = {}
            for p in ps:
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                runs.setdefault((p.device, int(st["step"].item())), []).append(p)
            b1, b2 = grp["betas"]
            for (dev, step), rps in runs.items():
                self._launch(dev, rps, float(grp["lr"]), float(b1), float(b2), float(grp["eps"]),
                             float(grp["weight_decay"]), step)
        return loss

    def _launch(self, dev, ps, lr, b1, b2, eps, wd, step):
        from . import _lib

        n = np.array([p.numel() for p in ps], dtype=np.int64)
        ptr = np.array([(p.data_ptr(), p.grad.data_ptr(), self.state[p]["exp_avg"].data_ptr(),
                         self.state[p]["exp_avg_sq"].data_ptr()) for p in ps], dtype=np.int64).reshape(-1, 4)
        nch = (n + CHUNK - 1) // CHUNK
        total = int(nch.sum())
        if total == 0:
            return
        idx = np.repeat(np.arange(len(ps)), nch)
        off = (np.arange(total) - np.repeat(np.cumsum(nch) - nch, nch)) * CHUNK
        rec = np.empty((total, 5), dtype=np.int64)   # include/pnr_abi.h pnr_adam_chunk: 4 pointers, n
        rec[:, :4] = ptr[idx] + (off * 4)[:, None]
        rec[:, 4] = np.minimum(CHUNK, n[idx] - off)
        nbytes = rec.nbytes
        if self._pinned is None or self._pinned.numel() < nbytes or self._table.device != dev:
            self._pinned = torch.empty(max(nbytes, 4096), dtype=torch.uint8, pin_memory=True)
            self._table = torch.empty(self._pinned.numel(), dtype=torch.uint8, device=dev)
            self._copied = None
        if self._copied is not None:
            self._copied.synchronize()   # the previous upload read the staging buffer (long done)
        self._pinned[:nbytes].numpy()[:] = np.frombuffer(rec.tobytes(), dtype=np.uint8)
        self._table[:nbytes].copy_(self._pinned[:nbytes], non_blocking=True)
        self._copied = torch.cuda.Event()
        self._copied.record(torch.cuda.current_stream(dev))
        _lib.check(_lib.load().pnr_adam_step(self._table.data_ptr(), total, lr, b1, b2, eps, wd, step,
                                             _lib.stream_of(dev)), "pnr_adam_step")
