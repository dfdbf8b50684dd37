"""ps_amd.ops -- hand-written HIP/CDNA4 kernels with thin torch wrappers.

GPU tensors always dispatch to ``ps_amd._C`` (raising if it is missing); CPU tensors use a
plain-torch reference implementation that doubles as the numerics oracle in tests.
"""
from ._ext import available, native, use_native  # noqa: F401
from . import optim, reduce, compress, sparse, nn_ops  # noqa: F401
from .optim import fused_opt, sparse_opt, SGD, ADAM, ADAGRAD, FTRL  # noqa: F401
