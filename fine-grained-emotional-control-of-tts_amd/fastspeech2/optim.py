"""Fused AdamW over the model's flat fp32 parameter / gradient buffers.

Same hyper-parameters and update rule as ``torch.optim.AdamW(model.parameters(), lr=lr)``
used by the reference (fastspeech2/train.py:232): betas (0.9, 0.999), eps 1e-8,
weight_decay 1e-2.  Scalars are computed in Python double exactly as torch's single-tensor
AdamW does, then one HBM-bound pass updates all 85.3 M parameters: ``fs2_adamw_prep`` when the
model's engine exists (the GEMM weights tile by tile, writing the next forward's bf16 weight
images from the updated values; the rest element-wise), else ``fs2_adamw``.
"""


import torch

from . import _native as N
from . import ops

# FS2_NO_FUSED_ADAMW=1: separate AdamW pass + weight-image pass at the next forward (A/B runs)
_NO_FUSED = N.exp_flag("FS2_NO_FUSED_ADAMW")


class FusedAdamW:
    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        self.model = model
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        model._ensure_packed()
        self.exp_avg = torch.zeros_like(model._flat)
        self.exp_avg_sq = torch.zeros_like(model._flat)
        self.step_count = 0

    def zero_grad(self, set_to_none=True):
        """Gradients accumulate into the flat buffer; zeroing it is one memset."""
        self.model._gflat.zero_()
        for n, p in self.model.named_parameters():
            p.grad = self.model._grad_views[n]

    def begin_step(self, grad_scale=1.0):
        """count the step and return its kernel scalars (torch single-tensor AdamW, double)"""
        self.step_count += 1
        b1, b2 = self.betas
        lr, wd, t = self.lr, self.weight_decay, self.step_count
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        return (1 - lr * wd, 1 - b1, b2, 1 - b2, lr / bc1, bc2 ** 0.5, self.eps, grad_scale)

    def fused_images(self):
        """the update can also write the engine's GEMM weight images (fs2_adamw_prep)"""
        m = self.model
        eng = m._engine
        return eng is not None and not _NO_FUSED and eng._flat_is(m._flat)

    @torch.no_grad()
    def step(self, grad_scale=1.0):
        m = self.model
        args = self.begin_step(grad_scale)
        eng = m._engine
        if self.fused_images():
            # the update also writes the next forward's GEMM weight images
            eng.adamw_step(self, *args)
            return
        ops.adamw(m._flat, m._gflat, self.exp_avg, self.exp_avg_sq, m._flat.numel(), *args)
        m.mark_params_updated()

    def _layout_record(self):
        """(name, offset, numel) of every parameter in the flat buffers the moments mirror"""
        return [(n, int(o), int(k)) for n, o, k, _, _ in self.model._layout]

    def state_dict(self):
        return {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "lr": self.lr, "betas": self.betas, "eps": self.eps,
                "weight_decay": self.weight_decay, "layout": self._layout_record()}

    def load_state_dict(self, sd):
        """moments saved under the same flat layout load as they are; saved under another
        layout (e.g. before a parameter-order change), each parameter's slice is moved to its
        current offset by name -- a state without a layout record is accepted only when the
        sizes match and no record says otherwise (older checkpoints of this layout)"""
        lay = sd.get("layout")
        cur = self._layout_record()
        if lay is None or [tuple(x) for x in lay] == cur:
            if sd["exp_avg"].numel() != self.exp_avg.numel():
                raise ValueError("FusedAdamW state: flat size mismatch and no layout record")
            self.exp_avg.copy_(sd["exp_avg"])
            self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        else:
            old = {n: (o, k) for n, o, k in lay}
            if set(old) != {n for n, _, _ in cur}:
                raise ValueError("FusedAdamW state: parameter names differ from this model's")
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            for n, o, k in cur:
                so, sk = old[n]
                if sk != k:
                    raise ValueError(f"FusedAdamW state: {n} has {sk} elements, model has {k}")
                self.exp_avg[o:o + k].copy_(sd["exp_avg"][so:so + k])
                self.exp_avg_sq[o:o + k].copy_(sd["exp_avg_sq"][so:so + k])
        self.step_count = sd["step"]
