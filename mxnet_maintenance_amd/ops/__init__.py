"""Operator library: registry + implementations (torch reference + gfx950 HIP kernels)."""
_loaded = False


def load_all():
    global _loaded
    if _loaded:
        return
    _loaded = True
    from . import tensor, nn, optimizer_ops, misc_ops, detection, quantization_ops, contrib_ops, control_flow, np_ops, transformer_ops, extra_ops, pdf_ops, fused_ops  # noqa: F401
