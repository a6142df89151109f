"""Record the ReLU branch the HIP kernels took after every BatchNorm2d.

The kernels apply BatchNorm+ReLU as relu(fmaf(y, scale, shift)) inside the
next conv's input load, and the backward keeps gz = g where
fmaf(y, scale, shift) > 0.  ainp_bn_relu_apply evaluates exactly that
expression, so applying it to the recorded pre-BatchNorm conv output with the
recorded (scale, shift) reproduces the kernels' mask bit for bit.  The masks
feed oracle.cnnblstm_ref.forward(relu_masks=...) (test infrastructure only).
"""
import contextlib

import torch.nn as nn


@contextlib.contextmanager
def recording(model):
    """with recording(model) as masks: <forward>  ->  masks {bn_name: bool cpu}"""
    from ainp import ops
    names = [n for n, m in model.named_modules() if isinstance(m, nn.BatchNorm2d)]
    masks = {}
    last = {}
    f_conv, f_fin, f_rfin = ops.conv3x3_fwd, ops.bn_finalize, ops.bn_reduce_finalize

    def conv(*a, **k):
        out = f_conv(*a, **k)
        y = out[0]
        if k.get("ycl"):                   # channel-last y [N, H, W, C] -> NCHW
            y = y.permute(0, 3, 1, 2)
        last["y"] = y.float().contiguous()     # bf16 storage: exact widening
        return out

    def record(out):
        sc, sh = out[0], out[1]
        name = names[len(masks)]
        masks[name] = (ops.bn_relu_apply(last["y"], sc, sh) > 0).cpu()
        return out

    def fin(*a, **k):          # data parallel: bn_finalize of the all-reduced sums
        return record(f_fin(*a, **k))

    def rfin(*a, **k):         # single process: the fused reduce + finalize
        return record(f_rfin(*a, **k))

    ops.conv3x3_fwd, ops.bn_finalize, ops.bn_reduce_finalize = conv, fin, rfin
    try:
        yield masks
    finally:
        ops.conv3x3_fwd, ops.bn_finalize, ops.bn_reduce_finalize = f_conv, f_fin, f_rfin
