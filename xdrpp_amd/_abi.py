"""ctypes binding of the C ABI declared in include/xdrgpu.h.

The shared library is built in-tree (xdrpp_amd/libxdrgpu.so, see
xdrpp_amd/build.py).  There is no fallback: if the library is missing the
import of anything that needs it raises, so a GPU run can never silently
take a CPU path.
"""
from __future__ import annotations

import ctypes as C
import os

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libxdrgpu.so")

# enum xdrg_op_kind
OP_U32, OP_U64, OP_BOOL, OP_ENUM, OP_OPAQUE, OP_VAROPAQUE, OP_STRING, OP_UNION, OP_JUMP, OP_END, OP_VECTOR = range(1, 12)
ABI_VERSION = 8  # XDRG_ABI_VERSION, include/xdrgpu.h
F_VALIDATE = 1
F_DEFAULT = 2
F_POINTER = 4
F_SUB = 8
SUB_FRAMES = 8  # XDRG_SUB_FRAMES (register frames of the element-subroutine walks' main pass)
MAX_FRAMES = 1 << 19  # XDRG_MAX_FRAMES

PATH_FIXED_REG, PATH_FIXED_LDS, PATH_VAR = 1, 2, 3

# enum xdrg_plan_option (xdrg_plan_set_option)
PLAN_OPTIONS = {"var_encode_kernel": 1, "var_decode_kernel": 2, "fixed_path": 3, "image_bytes": 4,
                "window_bytes": 5, "enc_unroll": 6, "dec_readahead": 7, "size_linear": 8,
                "grp_unroll": 9, "grp_blocks": 10, "grp_nontemporal": 11, "specialize": 12,
                "index_fast": 13, "stage_bytes": 14,
                "enc_stream": 15, "fixed_stream": 16}

OK = 0
API_ERRORS = {-1: "EINVAL", -2: "EALIGN", -3: "EUNSUPPORTED", -4: "EHIP", -5: "ENOMEM", -6: "ESPACE"}

# enum xdrg_err
ERR_NONE = 0
ERR_OVERFLOW_GET = 1
ERR_OVERFLOW_PUT = 2
ERR_XVECTOR_BOUND = 3
ERR_XSTRING_BOUND = 4
ERR_NONZERO_PAD = 5
ERR_BAD_DISCRIMINANT = 6
ERR_INVALID_ENUM = 7
ERR_STACK_PUT = 8
ERR_STACK_GET = 9
ERR_SIZE_NOT_MULT4 = 10
ERR_TRAILING = 11
ERR_POINTER_BOUND = 12
ERR_MSG_EOF = 13
ERR_MSG_SIZE4 = 14
ERR_MSG_FRAGMENT = 15
ERR_MSG_TOO_LONG = 16
ERR_MSG_MISMATCH = 17
ERR_MSG_COUNT = 18
ERR_LOOKBACK = 19
ERR_INDEX_LONG = 20

MARK_LAST = 0x80000000  # XDRG_MARK_LAST: last-fragment bit of a record mark
INDEX_MAX_MSG = 16380   # XDRG_INDEX_MAX_MSG (one list-ranking window)
MAX_MSG = 0x7FFFFFFF    # XDRG_MAX_MSG
MSG_SOCK_MAXMSGLEN = 0x100000  # msg_sock::default_maxmsglen, xdrpp/msgsock.h:29

XDR_MAX_LEN = 0xFFFFFFFC  # xdrpp/types.h:360
DEFAULT_STACK_LIMIT = 0xFFFFFFFF  # xdrpp/marshal.cc:6


class XdrgOp(C.Structure):
    _fields_ = [
        ("kind", C.c_uint8),
        ("flags", C.c_uint8),
        ("depth", C.c_uint16),
        ("noff", C.c_uint32),
        ("arg0", C.c_uint32),
        ("arg1", C.c_uint32),
        ("arg2", C.c_uint32),
        ("arg3", C.c_uint32),
        ("arg4", C.c_uint32),
        ("name", C.c_uint32),
    ]


assert C.sizeof(XdrgOp) == 32


class XdrgPlanInfo(C.Structure):
    _fields_ = [
        ("path", C.c_uint32),
        ("native_stride", C.c_uint32),
        ("fixed_size", C.c_uint32),
        ("max_depth", C.c_uint32),
        ("nops", C.c_uint32),
        ("has_checks", C.c_uint32),
        ("max_record_bytes", C.c_uint64),
        ("group_records", C.c_uint32),
        ("specialized", C.c_uint32),
    ]


class XdrgStatus(C.Structure):
    _fields_ = [("first_error", C.c_uint64), ("total_bytes", C.c_uint64)]


class XdrgError(C.Structure):
    _fields_ = [
        ("code", C.c_int32),
        ("exc", C.c_int32),
        ("record", C.c_uint64),
        ("op", C.c_uint32),
        ("rsv", C.c_uint32),
        ("total_bytes", C.c_uint64),
    ]


# Every symbol include/xdrgpu.h declares (checked by tests/test_abi.py).
EXPORTED = (
    "xdrg_abi_version", "xdrg_plan_create", "xdrg_plan_destroy", "xdrg_plan_get_info",
    "xdrg_workspace_size", "xdrg_status_init", "xdrg_status_read", "xdrg_encode",
    "xdrg_decode", "xdrg_serial_sizes", "xdrg_swap32", "xdrg_swap64",
    "xdrg_error_message", "xdrg_error_exception", "xdrg_last_hip_error",
    "xdrg_decode_heap_size", "xdrg_encode_msgs", "xdrg_decode_msgs", "xdrg_index_msgs",
    "xdrg_index_workspace_size", "xdrg_rpc_dispatch", "xdrg_rpc_check_replies",
    "xdrg_rpc_replies", "xdrg_rpc_replies_workspace_size", "xdrg_record_depths",
    "xdrg_plan_set_option", "xdrg_plan_kernel_source", "xdrg_plan_build_kernels",
    "xdrg_plan_load_kernels", "xdrg_index_records", "xdrg_encode_sizes", "xdrg_encode_sized",
    "xdrg_deep_workspace_size",
)

# RPC header batches (include/xdrgpu.h "RPC header batches")
RPC_DISPATCH, RPC_DROP_MALFORMED, RPC_DROP_NONCALL, RPC_RPC_MISMATCH, RPC_PROG_UNAVAIL, \
    RPC_PROG_MISMATCH, RPC_PROC_UNAVAIL, RPC_GARBAGE_ARGS, RPC_SYSTEM_ERR, RPC_AUTH_ERROR = range(10)
RPCR_OK, RPCR_ACCEPT_STAT, RPCR_AUTH_STAT, RPCR_RPCVERS_MISMATCH, RPCR_NOT_REPLY, RPCR_MALFORMED, \
    RPCR_BAD_XID = range(7)
RPC_W_RPCVERS, RPC_W_PROG, RPC_W_VERS, RPC_W_PROC, RPC_W_CRED_FLAVOR = range(5)
RPC_W_REPLY_STAT, RPC_W_STAT, RPC_W_WHY = range(3)
RPC_W_VERF_FLAVOR, RPC_W_LOW, RPC_W_HIGH = 5, 6, 7
RPC_PROC_IFACE_ONLY = 1
RPC_MAX_PROCS = 4096
RPC_HDR_BYTES = 64

_lib = None


class AbiError(RuntimeError):
    """An API-level failure (bad arguments, HIP error) of the C ABI."""


def lib() -> C.CDLL:
    """Load libxdrgpu.so (once).  Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (there is no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    vp, u64, u32, sz = C.c_void_p, C.c_uint64, C.c_uint32, C.c_size_t
    L.xdrg_abi_version.restype = C.c_int
    L.xdrg_plan_create.argtypes = [C.POINTER(XdrgOp), u32, C.POINTER(C.c_uint32), u32, u32, C.POINTER(vp)]
    L.xdrg_plan_create.restype = C.c_int
    L.xdrg_plan_destroy.argtypes = [vp]
    L.xdrg_plan_destroy.restype = None
    L.xdrg_plan_get_info.argtypes = [vp, C.POINTER(XdrgPlanInfo)]
    L.xdrg_plan_get_info.restype = C.c_int
    L.xdrg_plan_set_option.argtypes = [vp, C.c_int, C.c_int64]
    L.xdrg_plan_set_option.restype = C.c_int
    L.xdrg_plan_kernel_source.argtypes = [vp, C.c_char_p, sz, C.POINTER(sz)]
    L.xdrg_plan_kernel_source.restype = C.c_int
    L.xdrg_plan_build_kernels.argtypes = [vp]
    L.xdrg_plan_build_kernels.restype = C.c_int
    L.xdrg_plan_load_kernels.argtypes = [vp, vp, sz]
    L.xdrg_plan_load_kernels.restype = C.c_int
    L.xdrg_workspace_size.argtypes = [vp, u64]
    L.xdrg_workspace_size.restype = sz
    L.xdrg_deep_workspace_size.argtypes = [vp, u64]
    L.xdrg_deep_workspace_size.restype = sz
    L.xdrg_status_init.argtypes = [vp, vp]
    L.xdrg_status_init.restype = C.c_int
    L.xdrg_status_read.argtypes = [vp, vp, C.POINTER(XdrgError)]
    L.xdrg_status_read.restype = C.c_int
    L.xdrg_encode.argtypes = [vp, vp, u64, vp, u64, vp, u64, vp, u32, vp, sz, vp, vp]
    L.xdrg_encode.restype = C.c_int
    L.xdrg_decode.argtypes = [vp, vp, u64, vp, u64, vp, vp, u64, u32, vp, sz, vp, vp]
    L.xdrg_decode.restype = C.c_int
    L.xdrg_encode_msgs.argtypes = [vp, vp, u64, vp, u64, vp, u64, vp, u32, vp, sz, vp, vp]
    L.xdrg_encode_msgs.restype = C.c_int
    L.xdrg_encode_sizes.argtypes = [vp, vp, u64, vp, u64, u32, C.c_int, vp, sz, vp, vp]
    L.xdrg_encode_sizes.restype = C.c_int
    L.xdrg_encode_sized.argtypes = [vp, vp, u64, vp, u64, vp, u64, vp, u32, C.c_int, vp, sz, vp, vp]
    L.xdrg_encode_sized.restype = C.c_int
    L.xdrg_decode_msgs.argtypes = [vp, vp, u64, vp, u64, vp, vp, u64, u32, vp, sz, vp, vp]
    L.xdrg_decode_msgs.restype = C.c_int
    L.xdrg_index_msgs.argtypes = [vp, u64, u32, u64, vp, vp, vp, sz, vp, vp]
    L.xdrg_index_msgs.restype = C.c_int
    L.xdrg_index_records.argtypes = [vp, vp, u64, u64, u32, vp, vp, vp, sz, vp, vp]
    L.xdrg_index_records.restype = C.c_int
    L.xdrg_index_workspace_size.argtypes = [u64, u32]
    L.xdrg_index_workspace_size.restype = sz
    L.xdrg_rpc_dispatch.argtypes = [vp, u64, vp, u64, vp, u32, vp, vp]
    L.xdrg_rpc_dispatch.restype = C.c_int
    L.xdrg_rpc_check_replies.argtypes = [vp, u64, vp, u64, vp, vp, vp]
    L.xdrg_rpc_check_replies.restype = C.c_int
    L.xdrg_rpc_replies.argtypes = [vp, u64, vp, u64, vp, vp, sz, vp, vp]
    L.xdrg_rpc_replies.restype = C.c_int
    L.xdrg_rpc_replies_workspace_size.argtypes = [u64]
    L.xdrg_rpc_replies_workspace_size.restype = sz
    L.xdrg_record_depths.argtypes = [vp, vp, u64, vp, u64, vp, vp, sz, vp, vp]
    L.xdrg_record_depths.restype = C.c_int
    L.xdrg_serial_sizes.argtypes = [vp, vp, u64, vp, u64, vp, u32, vp, sz, vp, vp]
    L.xdrg_serial_sizes.restype = C.c_int
    L.xdrg_swap32.argtypes = [vp, vp, u64, vp]
    L.xdrg_swap32.restype = C.c_int
    L.xdrg_swap64.argtypes = [vp, vp, u64, vp]
    L.xdrg_swap64.restype = C.c_int
    L.xdrg_decode_heap_size.argtypes = [vp, u64]
    L.xdrg_decode_heap_size.restype = u64
    L.xdrg_error_message.argtypes = [C.c_int]
    L.xdrg_error_message.restype = C.c_char_p
    L.xdrg_error_exception.argtypes = [C.c_int]
    L.xdrg_error_exception.restype = C.c_int
    L.xdrg_last_hip_error.restype = C.c_char_p
    if L.xdrg_abi_version() != ABI_VERSION:
        raise ImportError("libxdrgpu.so ABI version mismatch")
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != OK:
        msg = API_ERRORS.get(rc, str(rc))
        if rc == -4:
            msg += ": " + lib().xdrg_last_hip_error().decode()
        raise AbiError(f"{what} failed: {msg}")
