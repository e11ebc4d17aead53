"""CPU tests of the RPC header batches.

The C restatement (oracle/xdr_oracle.c xdro_rpc_*) is pinned to what the
REAL reference produced (oracle/ref_golden rpc: reference xdr_get of each
rpc_msg header, rpc_server_base::dispatch's routing, check_call_hdr and the
server.cc reply builders over real message_t/xdr_put): server actions,
client statuses and error-reply bytes, bit-exact.  The dispatch workload
generator (xdrpp_amd.workloads.rpc_calls) is pinned to the committed input
stream and to the sha256 of the 1M-message stream.
"""
import collections
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLD, ROOT

from xdrpp_amd import _abi as A
from xdrpp_amd import rpc as R
from xdrpp_amd import workloads as W
import oracle_bridge as O

N = 1024


def g(name, dtype=np.uint8):
    return np.fromfile(os.path.join(GOLD, name), dtype=dtype)


def hdrs(name):
    return g(name).view(R.HDR_DTYPE)


def test_hdr_layout():
    assert R.HDR_DTYPE.itemsize == 64
    assert R.HDR_DTYPE.fields["w"][1] == 8
    assert R.HDR_DTYPE.fields["body_off"][1] == 48


def test_generator_matches_fixture(manifest):
    s, o = W.rpc_calls(N)
    assert np.array_equal(s, g(f"rpccall_{N}.stream"))
    assert np.array_equal(o, g(f"rpccall_{N}.msgoffs", "<u8"))
    assert np.array_equal(W.RPC_PROCS.astype("<u4").reshape(-1), g("rpc_procs.bin", "<u4"))


def test_generator_full_size_hash(manifest):
    h = manifest["hashes"]["rpccall_1048576"]
    s, _ = W.rpc_calls(1 << 20)
    assert s.size == h["stream_bytes"]
    assert hashlib.sha256(s.tobytes()).hexdigest() == h["stream"]


def test_index_of_call_stream():
    s = g(f"rpccall_{N}.stream")
    rc, cnt, offs = O.index_msgs(s, A.INDEX_MAX_MSG)
    assert (rc, cnt) == (0, N)
    assert np.array_equal(offs, g(f"rpccall_{N}.msgoffs", "<u8"))


def test_oracle_dispatch_matches_reference():
    s, o = g(f"rpccall_{N}.stream"), g(f"rpccall_{N}.msgoffs", "<u8")
    want = hdrs(f"rpccall_{N}.hdrs")
    got = O.rpc_headers(s, o, g("rpc_procs.bin", "<u4"))
    assert got.tobytes() == want.tobytes()
    # the workload reaches every route and every malformed-header error
    acts = collections.Counter(want["action"].tolist())
    assert set(acts) == {A.RPC_DISPATCH, A.RPC_DROP_MALFORMED, A.RPC_DROP_NONCALL,
                         A.RPC_RPC_MISMATCH, A.RPC_PROG_UNAVAIL, A.RPC_PROG_MISMATCH,
                         A.RPC_PROC_UNAVAIL}
    errs = set(want["err"].tolist())
    assert errs == {0, A.ERR_OVERFLOW_GET, A.ERR_XVECTOR_BOUND, A.ERR_NONZERO_PAD,
                    A.ERR_BAD_DISCRIMINANT}


def test_oracle_client_matches_reference():
    s, o = g(f"rpccall_{N}.stream"), g(f"rpccall_{N}.msgoffs", "<u8")
    assert O.rpc_headers(s, o, None, client=True).tobytes() == hdrs(f"rpccall_{N}.chk").tobytes()
    m, mo, x = g(f"rpc_{N}.msgs"), g(f"rpc_{N}.msgoffs", "<u8"), g(f"rpc_{N}.xids", "<u4")
    want = hdrs(f"rpc_{N}.chk")
    assert O.rpc_headers(m, mo, None, client=True, xids=x).tobytes() == want.tobytes()
    assert set(want["action"].tolist()) == {A.RPCR_OK, A.RPCR_ACCEPT_STAT, A.RPCR_AUTH_STAT,
                                            A.RPCR_RPCVERS_MISMATCH, A.RPCR_NOT_REPLY,
                                            A.RPCR_BAD_XID}


def test_oracle_replies_match_reference():
    h = hdrs(f"rpccall_{N}.hdrs")
    out, offs, rc, _ = O.rpc_replies(h)
    assert rc == 0
    assert out.tobytes() == g(f"rpccall_{N}.replies").tobytes()
    assert np.array_equal(offs, g(f"rpccall_{N}.replyoffs", "<u8"))


def test_oracle_auth_error_reply_known_answer():
    h = np.zeros(1, dtype=R.HDR_DTYPE)
    h["xid"], h["action"] = 0x01020304, A.RPC_AUTH_ERROR
    h["w"][0, A.RPC_W_WHY] = 5
    out, offs, rc, _ = O.rpc_replies(h)
    assert rc == 0 and out.tobytes() == g(f"rpccall_{N}.autherr").tobytes()


def test_oracle_replies_capacity():
    h = hdrs(f"rpccall_{N}.hdrs")
    full, offs, _, _ = O.rpc_replies(h)
    k = int(np.nonzero(np.diff(offs.astype(np.int64)) > 0)[0][3])  # 4th reply
    _, _, rc, er = O.rpc_replies(h, cap=int(offs[k]) + 4)
    assert (rc, er) == (A.ERR_OVERFLOW_PUT, k)


def test_proc_table_and_validation():
    t = R.proc_table({7: {2: [3, 1], 1: []}, 5: {1: [0]}})
    assert t.tolist() == [[5, 1, 0, 0], [7, 1, 0, A.RPC_PROC_IFACE_ONLY], [7, 2, 1, 0], [7, 2, 3, 0]]
    with pytest.raises(ValueError):
        R._check_table(t[::-1].copy())


def test_raise_for_reply_messages():
    h = np.zeros(1, dtype=R.HDR_DTYPE)[0]
    h["action"] = A.RPCR_OK
    R.raise_for_reply(h)
    cases = [(A.RPCR_ACCEPT_STAT, (A.RPC_W_STAT, 1), R.XdrCallError, "remote hasn't exported program"),
             (A.RPCR_AUTH_STAT, (A.RPC_W_WHY, 5), R.XdrCallError, "rejected for security reasons"),
             (A.RPCR_RPCVERS_MISMATCH, None, R.XdrCallError,
              "server reported rpcvers field with wrong value"),
             (A.RPCR_NOT_REPLY, None, R.XdrRuntimeError, "call received when reply expected"),
             (A.RPCR_BAD_XID, None, R.XdrRuntimeError, "synchronous_client: unexpected xid")]
    for act, w, cls, what in cases:
        h = np.zeros(1, dtype=R.HDR_DTYPE)[0]
        h["action"] = act
        if w:
            h["w"][w[0]] = w[1]
        with pytest.raises(cls) as ei:
            R.raise_for_reply(h)
        assert str(ei.value) == what


@pytest.mark.skipif(not os.path.exists("/root/reference/xdrpp/server.h"), reason="reference tree absent")
def test_success_fixture_regenerates(tmp_path):
    """success_rec128_512.{msgs,hdr7} are what the reference writes today
    (ref_golden success also asserts tests/arpc.cc:35-43: rpc_msg(7, REPLY)
    and rpc_success_hdr(7) marshal to the same message)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_ref/ref_golden"], check=True)
    pre = str(tmp_path / "s")
    subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ref_golden"), "success", "512", pre], check=True)
    for ext in ("msgs", "hdr7"):
        assert open(pre + "." + ext, "rb").read() == open(os.path.join(GOLD, "success_rec128_512." + ext), "rb").read()


def test_success_fixture_layout():
    """The fixture's messages: mark BE(152 | last), xid r * 2654435761,
    REPLY, MSG_ACCEPTED, AUTH_NONE, empty verf, SUCCESS, then 128 bytes."""
    m = g("success_rec128_512.msgs").reshape(512, 156)
    w = m[:, :28].copy().view(">u4")
    assert (w[:, 0] == (152 | A.MARK_LAST)).all()
    assert np.array_equal(w[:, 1], (np.arange(512, dtype=np.uint64) * 2654435761 & 0xFFFFFFFF).astype(np.uint32))
    assert (w[:, 2] == 1).all() and (w[:, 3:] == 0).all()
    assert g("success_rec128_512.hdr7").view(">u4").tolist() == [24 | A.MARK_LAST, 7, 1, 0, 0, 0, 0]
