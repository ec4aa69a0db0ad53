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
        # device chunk tables by (device, step run): rebuilt only when a pointer changes (the
        # caching allocator normally hands the gradients the same blocks every step); an upload
        # goes through a ring of pinned staging buffers, each reused only after its own copy
        # event -- never a wait on the current step's work, which would stop the host running ahead
        self._tables = {}
        self._ring, self._ring_i = [], 0

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
        key = (dev, ptr.tobytes(), n.tobytes())
        tab = self._tables.get(dev)
        if tab is None or tab[0] != key:
            nch = (n + CHUNK - 1) // CHUNK
            total = int(nch.sum())
            if total == 0:
                return
            idx = np.repeat(np.arange(len(ps)), nch)
            off = (np.arange(total) - np.repeat(np.cumsum(nch) - nch, nch)) * CHUNK
            rec = np.empty((total, 5), dtype=np.int64)   # include/pnr_abi.h pnr_adam_chunk: 4 pointers, n
            rec[:, :4] = ptr[idx] + (off * 4)[:, None]
            rec[:, 4] = np.minimum(CHUNK, n[idx] - off)
            raw = np.frombuffer(rec.tobytes(), dtype=np.uint8)
            dev_tab = torch.empty(raw.size, dtype=torch.uint8, device=dev)
            pinned, evt = self._stage(raw.size)
            pinned[:raw.size].numpy()[:] = raw
            dev_tab.copy_(pinned[:raw.size], non_blocking=True)
            evt.record(torch.cuda.current_stream(dev))
            tab = (key, dev_tab, total)
            self._tables[dev] = tab
        _lib.check(_lib.load().pnr_adam_step(tab[1].data_ptr(), tab[2], lr, b1, b2, eps, wd, step,
                                             _lib.stream_of(dev)), "pnr_adam_step")

    def _stage(self, nbytes):
        """A pinned staging buffer of the 4-slot ring, its previous upload finished."""
        if len(self._ring) < 4:
            self._ring.append([torch.empty(max(nbytes, 4096), dtype=torch.uint8, pin_memory=True), torch.cuda.Event()])
            slot = self._ring[-1]
        else:
            slot = self._ring[self._ring_i]
            self._ring_i = (self._ring_i + 1) % 4
            slot[1].synchronize()
            if slot[0].numel() < nbytes:
                slot[0] = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        slot[1] = torch.cuda.Event()
        return slot[0], slot[1]
