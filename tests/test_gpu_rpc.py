"""GPU parity of the RPC header batches through the C ABI:
xdrg_rpc_dispatch (rpc_server_base::dispatch routing), xdrg_rpc_check_replies
(check_call_hdr + xid test) and xdrg_rpc_replies (server.cc error replies).

Small batches are checked against what the REAL reference produced
(tests/golden/rpccall_1024.*, rpc_1024.chk); the 1M-message batch against
the reference's sha256 (manifest) and the C restatement; edge cases (empty
batches, bogus offsets, the global-memory registry path, output capacity)
against the C restatement, which tests/test_rpc.py pins to the fixtures.
Integer work: bit-exact.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLD

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from xdrpp_amd import _abi as A  # noqa: E402
from xdrpp_amd import marshal as M  # noqa: E402
from xdrpp_amd import rpc as R  # noqa: E402
from xdrpp_amd import schemas as S  # noqa: E402
from xdrpp_amd import workloads as W  # noqa: E402
import oracle_bridge as O  # noqa: E402

N = 1024


def g(name, dtype=np.uint8):
    return np.fromfile(os.path.join(GOLD, name), dtype=dtype)


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def offs_dev(o, dev):
    return to_dev(np.asarray(o, dtype=np.uint64).view(np.int64), dev)


def test_dispatch_golden(dev):
    s, o = g(f"rpccall_{N}.stream"), g(f"rpccall_{N}.msgoffs", "<u8")
    h = R.dispatch(to_dev(s, dev), offs_dev(o, dev), g("rpc_procs.bin", "<u4").reshape(-1, 4))
    assert h.cpu().numpy().tobytes() == g(f"rpccall_{N}.hdrs").tobytes()


def test_dispatch_on_device_index(dev):
    """index_messages -> dispatch, all on the device."""
    st = to_dev(g(f"rpccall_{N}.stream"), dev)
    offs = M.index_messages(st)
    h = R.dispatch(st, offs, g("rpc_procs.bin", "<u4").reshape(-1, 4))
    assert h.cpu().numpy().tobytes() == g(f"rpccall_{N}.hdrs").tobytes()


def test_check_replies_golden(dev):
    s, o = g(f"rpccall_{N}.stream"), g(f"rpccall_{N}.msgoffs", "<u8")
    h = R.check_replies(to_dev(s, dev), offs_dev(o, dev))
    assert h.cpu().numpy().tobytes() == g(f"rpccall_{N}.chk").tobytes()
    m, mo, x = g(f"rpc_{N}.msgs"), g(f"rpc_{N}.msgoffs", "<u8"), g(f"rpc_{N}.xids", "<u4")
    h = R.check_replies(to_dev(m, dev), offs_dev(mo, dev), to_dev(x.view(np.int32), dev))
    assert h.cpu().numpy().tobytes() == g(f"rpc_{N}.chk").tobytes()


def test_error_replies_golden(dev):
    h = to_dev(g(f"rpccall_{N}.hdrs"), dev)
    out, offs = R.error_replies(h)
    assert out.cpu().numpy().tobytes() == g(f"rpccall_{N}.replies").tobytes()
    assert np.array_equal(offs.cpu().numpy().view(np.uint64), g(f"rpccall_{N}.replyoffs", "<u8"))
    # the replies are a valid message stream (the client side reads them back)
    ro = M.index_messages(out)
    chk = R.hdrs_numpy(R.check_replies(out, ro))
    assert set(chk["action"].tolist()) <= {A.RPCR_ACCEPT_STAT, A.RPCR_RPCVERS_MISMATCH}


def test_auth_error_reply_known_answer(dev):
    h = np.zeros(3, dtype=R.HDR_DTYPE)
    h["action"] = [A.RPC_DISPATCH, A.RPC_AUTH_ERROR, A.RPC_DROP_NONCALL]
    h["xid"][1] = 0x01020304
    h["w"][1, A.RPC_W_WHY] = 5
    out, offs = R.error_replies(to_dev(h.view(np.uint8), dev))
    assert out.cpu().numpy().tobytes() == g(f"rpccall_{N}.autherr").tobytes()
    assert offs.cpu().tolist() == [0, 0, 24, 24]


def test_caller_set_actions(dev):
    """GARBAGE_ARGS / SYSTEM_ERR set by the caller after the args decode."""
    h = g(f"rpccall_{N}.hdrs").view(R.HDR_DTYPE).copy()
    d = np.nonzero(h["action"] == A.RPC_DISPATCH)[0]
    h["action"][d[::3]] = A.RPC_GARBAGE_ARGS
    h["action"][d[1::3]] = A.RPC_SYSTEM_ERR
    want, woffs, rc, _ = O.rpc_replies(h)
    out, offs = R.error_replies(to_dev(h.view(np.uint8), dev))
    assert rc == 0 and out.cpu().numpy().tobytes() == want.tobytes()
    assert np.array_equal(offs.cpu().numpy().view(np.uint64), woffs)


def test_replies_capacity(dev):
    h = g(f"rpccall_{N}.hdrs").view(R.HDR_DTYPE)
    _, woffs, _, _ = O.rpc_replies(h)
    k = int(np.nonzero(np.diff(woffs.astype(np.int64)) > 0)[0][5])
    cap = int(woffs[k]) + 8
    _, _, rc, er = O.rpc_replies(h, cap=cap)
    w = R.ReplyWriter(dev)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    offs = torch.empty(N + 1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    w.status.init(s)
    w.launch(to_dev(h.view(np.uint8), dev), out, offs, s)
    e = w.status.read(s)
    assert (e.code, e.record) == (rc, er) == (A.ERR_OVERFLOW_PUT, k)


def test_empty_batches(dev):
    s = torch.zeros(4, dtype=torch.uint8, device=dev)
    o = torch.zeros(1, dtype=torch.int64, device=dev)
    assert R.dispatch(s, o, W.RPC_PROCS).numel() == 0
    assert R.check_replies(s, o).numel() == 0
    out, offs = R.error_replies(torch.empty(0, dtype=torch.uint8, device=dev))
    assert out.numel() == 0 and offs.cpu().tolist() == [0]


def test_bogus_offsets_are_malformed(dev):
    s, o = g(f"rpccall_{N}.stream"), g(f"rpccall_{N}.msgoffs", "<u8").copy()
    o[5] = o[6] + 8      # message 5 ends before it starts, message 4 runs past 5's mark
    o[9] += 2            # misaligned mark
    o[-1] = s.size + 64  # past the stream
    want = O.rpc_headers(s, o, W.RPC_PROCS)
    got = R.hdrs_numpy(R.dispatch(to_dev(s, dev), offs_dev(o, dev), W.RPC_PROCS))
    assert got.tobytes() == want.tobytes()
    assert got["err"][5] == A.ERR_MSG_MISMATCH and got["action"][5] == A.RPC_DROP_MALFORMED


def test_large_registry_global_path(dev):
    """More procedures than the LDS stage holds (> 1024): table in global memory."""
    extra = np.array([(200000 + i // 40, 1 + (i // 8) % 5, i % 8, 0) for i in range(1600)],
                     dtype=np.uint32)
    t = np.concatenate([W.RPC_PROCS, extra])
    t = t[np.lexsort((t[:, 2], t[:, 1], t[:, 0]))]
    s, o = W.rpc_calls(1 << 14)
    want = O.rpc_headers(s, o, t)
    got = R.hdrs_numpy(R.dispatch(to_dev(s, dev), offs_dev(o, dev), t))
    assert got.tobytes() == want.tobytes()


def test_full_size(dev, manifest):
    h = manifest["hashes"]["rpccall_1048576"]
    s, o = W.rpc_calls(1 << 20)
    st, od = to_dev(s, dev), offs_dev(o, dev)
    hd = R.dispatch(st, od, W.RPC_PROCS)
    got = hd.cpu().numpy()
    assert hashlib.sha256(got.tobytes()).hexdigest() == h["hdrs"]
    ck = R.check_replies(st, od).cpu().numpy()
    assert hashlib.sha256(ck.tobytes()).hexdigest() == h["chk"]
    out, _ = R.error_replies(hd)
    assert hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest() == h["replies"]


def test_success_replies_are_xdr_to_msg(dev):
    """xdr_to_msg(rpc_success_hdr(xid), res): the success-reply record type
    through encode_msgs, against the argument-pack bytes (header words, then
    the result's encoding) and the client check reading them back as OK."""
    t = R.success_reply_type(S.rec128)
    p = M.Plan(t)
    n = 512
    res, _ = W.rec128(n)
    xid = (np.arange(n, dtype=np.uint32) * 2654435761).astype(np.uint32)
    nat = np.zeros((n, p.stride), dtype=np.uint8)
    hdr = np.zeros((n, 6), dtype="<u4")
    hdr[:, 0], hdr[:, 1] = xid, 1
    nat[:, :24] = hdr.view(np.uint8).reshape(n, 24)
    nat[:, 24:] = res.reshape(n, 128)
    enc = M.Marshaler(p, dev).encode_msgs(to_dev(nat.reshape(-1), dev), n)
    ref = M.Marshaler(M.Plan(S.rec128), dev).encode(to_dev(res, dev), n).xdr.cpu().numpy()
    words = np.zeros((n, 7), dtype=">u4")
    words[:, 0] = (24 + 128) | A.MARK_LAST
    words[:, 1], words[:, 2] = xid, 1
    want = np.concatenate([words.view(np.uint8).reshape(n, 28), ref.reshape(n, 128)], axis=1)
    assert np.array_equal(enc.xdr.cpu().numpy(), want.reshape(-1))
    chk = R.hdrs_numpy(R.check_replies(enc.xdr, enc.offsets, to_dev(xid.view(np.int32), dev)))
    assert (chk["action"] == A.RPCR_OK).all()
    assert np.array_equal(chk["body_off"], enc.offsets.cpu().numpy()[:-1].astype(np.uint64) + 28)


def test_success_replies_match_reference(dev):
    """xdr_to_msg(rpc_success_hdr(xid), res) as the REAL reference writes it
    (tests/golden/success_rec128_512.msgs from oracle/ref_golden success:
    xdrpp/server.h:27-49, the reply srpc_service::dispatch sends at
    srpc.h:152) equals encode_msgs of the success-reply record type; and the
    header alone equals the reference's rpc_success_hdr(7) message, which
    ref_golden asserts is rpc_msg(7, REPLY)'s (tests/arpc.cc:35-43)."""
    n = 512
    want = np.fromfile(os.path.join(GOLD, f"success_rec128_{n}.msgs"), dtype=np.uint8)
    t = R.success_reply_type(S.rec128)
    p = M.Plan(t)
    res, _ = W.rec128(n)
    xid = (np.arange(n, dtype=np.uint64) * 2654435761 & 0xFFFFFFFF).astype(np.uint32)
    nat = np.zeros((n, p.stride), dtype=np.uint8)
    hdr = np.zeros((n, 6), dtype="<u4")
    hdr[:, 0], hdr[:, 1] = xid, 1  # xid, REPLY (MSG_ACCEPTED, AUTH_NONE, empty body, SUCCESS: 0)
    nat[:, :24] = hdr.view(np.uint8).reshape(n, 24)
    nat[:, 24:] = res.reshape(n, 128)
    enc = M.Marshaler(p, dev).encode_msgs(to_dev(nat.reshape(-1), dev), n)
    assert np.array_equal(enc.xdr.cpu().numpy(), want)
    h7 = np.fromfile(os.path.join(GOLD, f"success_rec128_{n}.hdr7"), dtype=np.uint8)
    hdr_t = S.Struct("rpc_success_hdr", [(f, S.UInt) for f in ("xid", "mtype", "stat", "flavor", "body", "accept")])
    one = np.array([7, 1, 0, 0, 0, 0], dtype="<u4").view(np.uint8)
    got7 = M.Marshaler(M.Plan(hdr_t), dev).encode_msgs(to_dev(one, dev), 1).xdr.cpu().numpy()
    assert np.array_equal(got7, h7)


@pytest.mark.parametrize("seed", range(4))
def test_fuzzed_headers_vs_oracle(dev, seed):
    """Random word corruptions of the call stream (lengths, discriminants,
    pads, flavors) and random message lengths: every header's route,
    client status and error replies equal the C restatement."""
    rng = np.random.default_rng(1234 + seed)
    s, o = W.rpc_calls(3000, first=7 * seed)
    s = s.copy()
    w = s.view("<u4")
    marks = (o[:-1] // 4).astype(np.int64)
    for _ in range(1500):  # corrupt header words (never the marks)
        k = int(rng.integers(0, len(marks)))
        pos = int(marks[k] + 1 + rng.integers(0, 12))
        if pos >= len(w) or pos in set(marks[k:k + 2].tolist()):
            continue
        w[pos] = np.uint32(rng.choice([0, 1, 2, 3, 400, 401, 0xFFFFFFFF,
                                       int(rng.integers(0, 1 << 32))])).byteswap()
    # some messages cut short: move an offset down (the index would reject
    # such framing; dispatch sees the shorter message and must not read past it)
    o2 = o.copy()
    for k in rng.integers(1, len(o) - 1, size=50):
        o2[k] = max(o2[k - 1] + 4, o2[k] - 4 * int(rng.integers(1, 8)))
    t = W.RPC_PROCS
    want = O.rpc_headers(s, o2, t)
    got = R.hdrs_numpy(R.dispatch(to_dev(s, dev), offs_dev(o2, dev), t))
    assert got.tobytes() == want.tobytes()
    wc = O.rpc_headers(s, o2, None, client=True)
    gc = R.hdrs_numpy(R.check_replies(to_dev(s, dev), offs_dev(o2, dev)))
    assert gc.tobytes() == wc.tobytes()
    rs, roffs, rc, _ = O.rpc_replies(want)
    out, goffs = R.error_replies(to_dev(want.view(np.uint8), dev))
    assert rc == 0 and out.cpu().numpy().tobytes() == rs.tobytes()
    assert np.array_equal(goffs.cpu().numpy().view(np.uint64), roffs)
