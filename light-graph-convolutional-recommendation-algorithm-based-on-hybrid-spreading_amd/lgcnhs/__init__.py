"""lgcnhs — MI355X-native hot path of LGCNHS (LightGCN propagation, hybrid spreading,
full-catalog masked top-K) behind the reference's Python API.

The HIP kernels live in ``csrc/`` and are reached through the C ABI of
``include/lgcnhs.h`` (``lib/liblgcnhs.so``); ``ops`` wraps them for torch tensors and the
``model/``, ``utils/`` mirror modules next to this package keep the reference's
function names and signatures.
"""
from .build import build_native  # noqa: F401
