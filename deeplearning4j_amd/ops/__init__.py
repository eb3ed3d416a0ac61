"""Array-engine ops: the slice of ND4J/libnd4j + cuDNN that the model layer calls.

Each op dispatches to a hand-written gfx950 HIP kernel on GPU tensors (``ops.native``) and to a
plain-torch reference on CPU tensors. See ``dispatch`` for the policy knobs.
"""
from .conv import conv2d_backward, conv2d_forward, conv_transpose2d_forward, depthwise_conv2d_forward
from .dispatch import native_enabled, native_lib, use_native
from .loss import softmax_xent
from .norm import bn_backward, bn_forward, bn_pool_backward, bn_pool_forward, layer_norm_backward, layer_norm_forward
from .pool import pool2d_backward, pool2d_forward
from .update import Segment, UpdatePlan, fused_update

__all__ = ["conv2d_forward", "conv2d_backward", "conv_transpose2d_forward", "depthwise_conv2d_forward",
           "pool2d_forward", "pool2d_backward", "bn_forward", "bn_backward", "bn_pool_forward", "bn_pool_backward",
           "layer_norm_forward", "layer_norm_backward", "softmax_xent", "fused_update", "UpdatePlan", "Segment", "native_lib",
           "use_native", "native_enabled"]
