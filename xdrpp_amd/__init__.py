"""xdrpp_amd — MI355X-native batched XDR (RFC 4506) marshal engine.

Accelerates xdrpp's encode/decode hot path (xdr_put / xdr_get,
xdr_to_opaque / xdr_from_opaque, xdrpp/marshal.{h,cc}; swap32,
xdrpp/endian.h) with hand-written gfx950 HIP kernels behind a C ABI
(include/xdrgpu.h).  Python pieces:

  xdr_types   descriptors mirroring the xdrc-generated types + plan compiler
  schemas     the benchmark schemas (numerics, rec128, recvar, rpc_msg)
  marshal     torch-facing batch API with the reference's exception types
  workloads   deterministic synthetic batches
  build       hipcc build of libxdrgpu.so (in-tree)
"""
from . import xdr_types, schemas  # noqa: F401  (no GPU needed)

__all__ = ["xdr_types", "schemas", "marshal", "workloads", "build"]
