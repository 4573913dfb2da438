"""sproxy_amd -- MI355X-native batched MD5 for sproxy's chunk checksum path.

The product is libmd5hip.so (sproxy_amd/csrc, C ABI in include/); this package
is the Python host mirror of that ABI (sproxy_amd.md5).
"""
from .md5 import (MD5Context, MD5Init, MD5Update, MD5Final, MD5_DIGEST_SIZE,  # noqa: F401
                  MD5HipError, digest_fixed, digest_desc, plan_order, fill_synthetic,
                  Batcher, variant_name, VARIANTS)

__version__ = "0.1.0"
