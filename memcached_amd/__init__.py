"""memcached_amd -- MI355X-native batched CRC-32C for memcached's extstore path.

The product is the C-ABI library ``libmcrc32c.so`` (include/crc32c.h drop-in +
include/crc32c_batch.h).  This package builds it (``memcached_amd.build``),
binds it (``memcached_amd.crc32c``) and mirrors the item layout the CRC spans
cover (``memcached_amd.layout``).
"""
__all__ = ["build", "layout", "crc32c"]
