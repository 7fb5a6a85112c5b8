"""Parameter containers with the reference's exact state-dict layout.

The modules built here only hold parameters and buffers (so ``state_dict``,
``load_state_dict``, ``parameters``, ``train``/``eval`` and checkpoint files
behave exactly like the reference's); inference runs in the HIP engine.
"""
import torch
import torch.nn as nn


class _Node(nn.Module):
    pass


def build_param_tree(root, shapes, buffers=("running_mean", "running_var",
                                             "num_batches_tracked")):
    """Create nested sub-modules on ``root`` so that its state_dict keys are
    exactly ``[k for k, _ in shapes]`` (in that order)."""
    for key, shape in shapes:
        parts = key.split(".")
        mod = root
        for p in parts[:-1]:
            if not hasattr(mod, p) or not isinstance(getattr(mod, p), nn.Module):
                mod.add_module(p, _Node())
            mod = getattr(mod, p)
        leaf = parts[-1]
        if leaf in buffers:
            dtype = torch.long if leaf == "num_batches_tracked" else torch.float32
            mod.register_buffer(leaf, torch.zeros(shape, dtype=dtype))
        else:
            mod.register_parameter(leaf, nn.Parameter(torch.zeros(shape)))
    return root
