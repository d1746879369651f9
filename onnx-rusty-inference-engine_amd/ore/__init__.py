"""ore — MI355X-native (gfx950) fp32 ONNX op executor for the op path of
jackperlo/onnx-rusty-inference-engine.  Python host mirror over the C ABI in include/ore.h;
all compute runs as HIP kernels in lib/libore.so (no CPU fallback)."""
from ._lib import (CONV_ALGO_DIRECT, CONV_ALGO_WINOGRAD, FUSE_ALIAS, FUSE_ALL, FUSE_CONCAT, FUSE_CONCAT_POOL,  # noqa: F401
                   FUSE_CONV_POOL, FUSE_CONV_RELU, FUSE_EAGER, FUSE_FIRE, FUSE_FIRE_POOL, FUSE_FIRST_SQUEEZE,
                   FUSE_POOL_SQUEEZE, FUSE_CONV_GAP, FUSE_POOL_EXPAND, KEEP_VALUES, LIB_PATH, LOAD_F16, LOAD_NO_WINOGRAD, OreError,
                   ABI_VERSION,
                   load)
from .engine import (Context, Model, add, concatenation, conv_out_shape, convolution, drop_out,  # noqa: F401
                     global_average_pool, inference, max_pool, mul, pool_out_shape, relu, reshape, softmax)

__version__ = "0.1.0"
