"""CPU: record-marked message batches (message_t, RFC 5531 record marking).

The fixtures tests/golden/<schema>_<n>.msgs / .msgoffs are what the REAL
reference produced: xdr_to_msg(r) per record (xdrpp/marshal.h:252-260),
whose mark message_t::alloc writes (xdrpp/marshal.cc:15-31), raw_data() of
raw_size() bytes each, back to back; ref_golden also read every message
back with xdr_from_msg.  These tests pin the C restatement (oracle/
xdr_oracle.c: xdro_encode_msgs / xdro_decode_msgs / xdro_index_msgs) to
them, so it can check the GPU on inputs no fixture covers.

The framing checks of the index (read_message, xdrpp/srpc.cc:29-55;
msg_sock's maxmsglen_, xdrpp/msgsock.cc:85-111) cannot be run from the
reference here: srpc.cc and msgsock.cc need xdrc's rpc_msg.hh, which
needs the xdrc front end (bison/flex, absent).  Their error cases below are
restated from those lines -- parity for framing errors is "unpinned" by a
reference run; parity for well-formed streams is pinned by the fixtures.
No GPU is used.
"""
import hashlib

import numpy as np
import pytest

from conftest import SMALL_N, golden

import oracle_bridge as O
from xdrpp_amd import _abi as A
from xdrpp_amd import marshal as M
from xdrpp_amd import schemas as S
from xdrpp_amd import workloads as W
from xdrpp_amd.xdr_types import compile_plan

SCHEMAS = ["numerics", "rec128", "recvar", "rpc", "vecrec", "containertest"]
CP = {k: compile_plan(t) for k, t in S.ALL.items()}


def mark(size: int, last: bool = True) -> bytes:
    return ((size | (A.MARK_LAST if last else 0)) & 0xFFFFFFFF).to_bytes(4, "big")


def stream(*parts: bytes) -> np.ndarray:
    return np.frombuffer(b"".join(parts), dtype=np.uint8).copy()


@pytest.mark.parametrize("name", SCHEMAS)
def test_oracle_encode_msgs_equals_reference(name):
    n = SMALL_N[name]
    x, offs = O.encode_msgs(CP[name], golden(name, n, "native"), n, golden(name, n, "heap"))
    assert np.array_equal(x, golden(name, n, "msgs"))
    assert np.array_equal(offs, golden(name, n, "msgoffs", np.uint64))


@pytest.mark.parametrize("name", SCHEMAS)
def test_reference_messages_are_marks_plus_records(name):
    """Message r = BE(size | 0x80000000) + the record's xdr_to_opaque bytes."""
    n = SMALL_N[name]
    m, mo = golden(name, n, "msgs"), golden(name, n, "msgoffs", np.uint64)
    x, xo = golden(name, n, "xdr"), golden(name, n, "offsets", np.uint64)
    for r in range(0, n, 97):
        body = x[xo[r]:xo[r + 1]]
        assert m[mo[r]:mo[r] + 4].tobytes() == mark(body.size)
        assert np.array_equal(m[mo[r] + 4:mo[r + 1]], body)
    assert mo[n] == m.size == x.size + 4 * n


@pytest.mark.parametrize("name", SCHEMAS)
def test_oracle_index_of_reference_stream(name):
    n = SMALL_N[name]
    rc, cnt, offs = O.index_msgs(golden(name, n, "msgs"), A.INDEX_MAX_MSG)
    assert (rc, cnt) == (0, n)
    assert np.array_equal(offs, golden(name, n, "msgoffs", np.uint64))


@pytest.mark.parametrize("name", SCHEMAS)
def test_oracle_decode_msgs_round_trip(name):
    n = SMALL_N[name]
    m, mo = golden(name, n, "msgs"), golden(name, n, "msgoffs", np.uint64)
    nat, heap = O.decode_msgs(CP[name], m, n, mo)
    if not CP[name].is_var:
        assert np.array_equal(nat, golden(name, n, "native"))
    x2, o2 = O.encode_msgs(CP[name], nat, n, heap)
    assert np.array_equal(x2, m) and np.array_equal(o2, mo)


def test_known_answer_message(kat):
    nat, _ = W.numerics(1)
    x, _ = O.encode_msgs(CP["numerics"], nat, 1)
    assert x.tobytes().hex() == kat["numerics_msg"]


@pytest.mark.parametrize("key", ["recvar_65536", "rpc_65536", "vecrec_65536", "numerics_65536"])
def test_oracle_msgs_manifest(manifest, key):
    name, n = key.rsplit("_", 1)
    n = int(n)
    nat, heap = W.GENERATORS[name](n)
    x, offs = O.encode_msgs(CP[name], nat, n, heap)
    h = manifest["hashes"][key]
    assert hashlib.sha256(x.tobytes()).hexdigest() == h["msgs"]
    assert hashlib.sha256(offs.tobytes()).hexdigest() == h["msgoffs"]


# ------------------------------------------- framing (read_message order)
FRAMING = {
    # name: (stream bytes, max_msg_len, max_msgs, expected rc, count)
    "empty": (b"", 64, None, 0, 0),
    "one": (mark(8) + b"\0" * 8, 64, None, 0, 1),
    "zero_length_messages": (mark(0) * 5, 64, None, 0, 5),
    "eof_in_mark": (mark(4) + b"\0" * 4 + b"\x80\0", 64, None, A.ERR_MSG_EOF, 1),
    "eof_in_body": (mark(4) + b"\0" * 4 + mark(12) + b"\0" * 8, 64, None, A.ERR_MSG_EOF, 1),
    "fragment_bit_clear": (mark(4) + b"\0" * 4 + mark(4, last=False) + b"\0" * 4, 64, None,
                           A.ERR_MSG_FRAGMENT, 1),
    # the pre-swap test (srpc.cc:38-39) reads the mark's first byte on this host
    "size_bits_24_25": (mark(0x01000004) + b"\0" * 4, 64, None, A.ERR_MSG_SIZE4, 0),
    "too_long": (mark(4) + b"\0" * 4 + mark(68) + b"\0" * 68, 64, None, A.ERR_MSG_TOO_LONG, 1),
    "size_not_mult4": (mark(4) + b"\0" * 4 + mark(5) + b"\0" * 8, 64, None,
                       A.ERR_SIZE_NOT_MULT4, 1),
    "count_limit": (mark(0) * 5, 64, 3, A.ERR_MSG_COUNT, 3),
    "count_limit_exact": (mark(0) * 3, 64, 3, 0, 3),
}


@pytest.mark.parametrize("case", list(FRAMING))
def test_oracle_framing(case):
    data, maxlen, maxm, want_rc, want_cnt = FRAMING[case]
    s = stream(data)
    rc, cnt, offs = O.index_msgs(s, maxlen, maxm)
    assert (rc, cnt) == (want_rc, want_cnt)
    # offsets: every mark before the stop, then the stop position
    pos, expect = 0, []
    for _ in range(cnt):
        expect.append(pos)
        pos += 4 + (int.from_bytes(data[pos:pos + 4], "big") & 0x7FFFFFFF)
    expect.append(pos)
    assert offs.tolist() == expect


@pytest.mark.parametrize("code,what", [
    (A.ERR_MSG_EOF, "read_message: premature EOF"),
    (A.ERR_MSG_SIZE4, "read_message: received size not multiple of 4"),
    (A.ERR_MSG_FRAGMENT, "read_message: message fragments unimplemented"),
    (A.ERR_MSG_TOO_LONG, "msg_sock: rejecting message (too long)"),
    (A.ERR_MSG_MISMATCH, "record mark does not match the record index"),
    (A.ERR_MSG_COUNT, "more messages than the record index holds"),
])
def test_framing_errors_map_to_bad_message_size(code, what):
    """read_message throws xdr_bad_message_size (srpc.cc:36-52)."""
    plan = M.Plan(CP["recvar"])  # host-only
    err = A.XdrgError(code=code, exc=0, record=7, op=0xFFFFFFFF, rsv=0, total_bytes=0)
    exc = M.error_from(plan, err)
    assert type(exc) is M.XdrBadMessageSize
    assert str(exc) == what and exc.record == 7 and exc.op is None


def test_oracle_decode_msgs_checks_marks():
    cp = CP["recvar"]
    n = 8
    m = golden("recvar", SMALL_N["recvar"], "msgs")
    mo = golden("recvar", SMALL_N["recvar"], "msgoffs", np.uint64)[:n + 1].copy()
    m = m[:int(mo[n])].copy()
    O.decode_msgs(cp, m, n, mo)
    bad = m.copy()
    bad[mo[3]] &= 0x7F  # record 3: fragment bit cleared
    with pytest.raises(O.OracleError) as ei:
        O.decode_msgs(cp, bad, n, mo)
    assert (ei.value.code, ei.value.record) == (A.ERR_MSG_FRAGMENT, 3)
    bad = m.copy()
    bad[mo[5] + 3] ^= 4  # record 5: mark size disagrees with the index
    with pytest.raises(O.OracleError) as ei:
        O.decode_msgs(cp, bad, n, mo)
    assert (ei.value.code, ei.value.record) == (A.ERR_MSG_MISMATCH, 5)
