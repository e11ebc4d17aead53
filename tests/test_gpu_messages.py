"""GPU parity of record-marked message batches (message_t, RFC 5531), through
the C ABI: xdrg_encode_msgs (= xdr_to_msg per record), xdrg_decode_msgs
(= xdr_from_msg per message) and xdrg_index_msgs (the record-mark framing
of read_message / msg_sock::input, found on the device by list ranking).

Well-formed streams are checked against the bytes the REAL reference
produced (tests/golden/*.msgs, *.msgoffs, manifest sha256); framing errors
and fuzzed streams against the C restatement (oracle/xdr_oracle.c), which
tests/test_messages.py pins to those fixtures.  Integer work: bit-exact.
"""
import hashlib

import numpy as np
import pytest

from conftest import SMALL_N, golden

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from xdrpp_amd import _abi as A  # noqa: E402
from xdrpp_amd import marshal as M  # noqa: E402
from xdrpp_amd import schemas as S  # noqa: E402
from xdrpp_amd import workloads as W  # noqa: E402
import oracle_bridge as O  # noqa: E402

SCHEMAS = ["numerics", "rec128", "recvar", "rpc", "vecrec", "containertest", "rp_list"]
_plans = {}


def plan(name, **options):
    """The plan of a schema, with launch options (xdrg_plan_set_option)."""
    key = (name, tuple(sorted(options.items())))
    if key not in _plans:
        _plans[key] = M.Plan(S.ALL[name], options)
    return _plans[key]


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def mark(size, last=True):
    return ((size | (A.MARK_LAST if last else 0)) & 0xFFFFFFFF).to_bytes(4, "big")


def gpu_index(x, dev, maxlen, max_msgs=None):
    """(rc, count, offsets[:count+1]) from the device, like O.index_msgs."""
    t = to_dev(x, dev) if x.size else torch.empty(0, dtype=torch.uint8, device=dev)
    try:
        offs = M.index_messages(t, maxlen, max_msgs)
        return 0, offs.numel() - 1, offs.cpu().numpy().view(np.uint64)
    except M.XdrRuntimeError as e:
        return e.code, e.record, None


def check_index(x, dev, maxlen, max_msgs=None):
    want = O.index_msgs(x, maxlen, max_msgs)
    got = gpu_index(x, dev, maxlen, max_msgs)
    assert got[:2] == want[:2]
    if got[0] == 0:
        assert np.array_equal(got[2], want[2])
    return want


# ---------------------------------------------------------------- golden
@pytest.mark.parametrize("name", SCHEMAS)
def test_encode_msgs_golden(dev, name):
    n = SMALL_N[name]
    mar = M.Marshaler(plan(name), dev)
    heap = golden(name, n, "heap")
    res = mar.encode_msgs(to_dev(golden(name, n, "native"), dev), n,
                          to_dev(heap, dev) if heap.size else None)
    assert np.array_equal(res.xdr.cpu().numpy(), golden(name, n, "msgs"))
    assert np.array_equal(res.offsets.cpu().numpy().view(np.uint64), golden(name, n, "msgoffs", np.uint64))


@pytest.mark.parametrize("name", SCHEMAS)
def test_index_of_reference_stream(dev, name):
    n = SMALL_N[name]
    rc, cnt, offs = gpu_index(golden(name, n, "msgs"), dev, A.INDEX_MAX_MSG)
    assert (rc, cnt) == (0, n)
    assert np.array_equal(offs, golden(name, n, "msgoffs", np.uint64))


@pytest.mark.parametrize("name", SCHEMAS)
@pytest.mark.parametrize("indexed", [True, False])
def test_decode_msgs_golden(dev, name, indexed):
    n = SMALL_N[name]
    p = plan(name)
    mar = M.Marshaler(p, dev)
    m, mo = golden(name, n, "msgs"), golden(name, n, "msgoffs", np.uint64)
    nat, heap = mar.decode_msgs(to_dev(m, dev), n if indexed else None,
                                to_dev(mo.view(np.int64), dev) if indexed else None)
    o_nat, o_heap = O.decode_msgs(p.cp, m, n, mo)
    assert np.array_equal(nat.cpu().numpy(), o_nat)
    if p.is_fixed:
        assert np.array_equal(nat.cpu().numpy(), golden(name, n, "native"))
    else:
        assert np.array_equal(heap.cpu().numpy(), o_heap)
        res = mar.encode_msgs(nat, n, heap)  # decode -> encode reproduces the reference
        assert np.array_equal(res.xdr.cpu().numpy(), m)


def test_known_answer_message(dev, kat):
    mar = M.Marshaler(plan("numerics"), dev)
    nat, _ = W.numerics(1)
    assert mar.encode_msgs(to_dev(nat, dev), 1).xdr.cpu().numpy().tobytes().hex() == kat["numerics_msg"]


# ------------------------------------------------------------- full size
@pytest.mark.parametrize("name,n", [("recvar", 1 << 20), ("rpc", 1 << 20), ("rec128", 1 << 20),
                                    ("vecrec", 1 << 16), ("numerics", 1 << 16)])
def test_full_size_msgs(dev, manifest, name, n):
    """Reference sha256 of the 1M-message stream; the device index of it
    equals the encoder's offsets (a multi-level index: 12K+ segments); and
    decode -> encode is the identity on the wire."""
    h = manifest["hashes"][f"{name}_{n}"]
    p = plan(name)
    mar = M.Marshaler(p, dev)
    nat, heap = W.GENERATORS[name](n)
    res = mar.encode_msgs(to_dev(nat, dev), n, to_dev(heap, dev) if heap.size else None)
    assert hashlib.sha256(res.xdr.cpu().numpy().tobytes()).hexdigest() == h["msgs"]
    assert hashlib.sha256(res.offsets.cpu().numpy().tobytes()).hexdigest() == h["msgoffs"]
    maxlen = min(p.max_record_bytes, A.INDEX_MAX_MSG)
    idx = M.index_messages(res.xdr, maxlen)
    assert torch.equal(idx, res.offsets)
    back, bheap = mar.decode_msgs(res.xdr, n, idx)
    if p.is_fixed:
        assert torch.equal(back, to_dev(nat, dev))
    else:
        assert torch.equal(mar.encode_msgs(back, n, bheap).xdr, res.xdr)


# --------------------------------------------------------- framing cases
def _stream(parts):
    return np.frombuffer(b"".join(parts), dtype=np.uint8).copy()


SEG = 16384  # bytes per index segment (kIxSW words)


def _messages(sizes, fill=0x5A):
    return _stream([mark(int(s)) + bytes([fill]) * int(s) for s in sizes])


@pytest.mark.parametrize("case", [
    "empty", "zero_length", "one_segment_exact", "spans_segments", "max_len_chain",
    "eof_in_mark", "eof_in_body", "fragment", "size_bits", "too_long", "mult4", "count"])
def test_index_framing_vs_oracle(dev, case):
    rng = np.random.default_rng(7)
    maxlen = 1024
    if case == "empty":
        x = _stream([])
    elif case == "zero_length":  # every word a mark: 4096 marks per segment
        x = _messages([0] * 20000)
    elif case == "one_segment_exact":  # the end falls exactly on a segment boundary
        x = _messages([SEG - 4])
        maxlen = A.INDEX_MAX_MSG
    elif case == "spans_segments":
        x = _messages(list(rng.integers(0, 256, 3000) * 4))
    elif case == "max_len_chain":
        x = _messages([maxlen] * 200)
    elif case == "eof_in_mark":
        x = np.concatenate([_messages([8] * 1000), _stream([b"\x80\x00"])])
    elif case == "eof_in_body":
        x = np.concatenate([_messages([8] * 5000), _stream([mark(40) + b"\0" * 12])])
    elif case == "fragment":
        x = _stream([mark(8) + b"\0" * 8] * 3000 + [mark(8, False) + b"\0" * 8] + [mark(0)] * 10)
    elif case == "size_bits":
        x = _stream([mark(4) + b"\0" * 4] * 4500 + [mark(0x02000000) + b"\0" * 4])
    elif case == "too_long":
        x = _messages([16] * 7000 + [maxlen + 4] + [0] * 3)
    elif case == "mult4":
        x = _stream([mark(12) + b"\0" * 12] * 2000 + [mark(6) + b"\0" * 8] + [mark(0)] * 4)
    else:  # more messages than the index holds
        x = _messages([4] * 9000)
        check_index(x, dev, maxlen, max_msgs=8191)
        return
    check_index(x, dev, maxlen)


@pytest.mark.parametrize("sizes", ["mixed", "zero", "max"])
def test_index_walk_holds(dev, sizes):
    """Well-framed streams of several segments: the speculative walk over the
    marks (index_kernels.h mark_rx) holds the index itself -- its flag, the
    first u32 of the workspace's last 256 bytes -- and equals the oracle's;
    every word a mark (zero-length messages) and maximal messages included."""
    rng = np.random.default_rng(11)
    maxlen = 1024
    sz = {"mixed": list(rng.integers(0, 257, 6000) * 4), "zero": [0] * 40000, "max": [maxlen] * 400}[sizes]
    x = _messages(sz)
    want = O.index_msgs(x, maxlen, None)
    L = A.lib()
    t = to_dev(x, dev)
    ws = torch.empty(L.xdrg_index_workspace_size(x.size, maxlen), dtype=torch.uint8, device=dev)
    offs = torch.empty(len(sz) + 1, dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    st = M.Status(dev)
    s = torch.cuda.current_stream().cuda_stream
    st.init(s)
    A.check(L.xdrg_index_msgs(t.data_ptr(), x.size, maxlen, len(sz), offs.data_ptr(), cnt.data_ptr(),
                              ws.data_ptr(), ws.numel(), st.ptr, s), "xdrg_index_msgs")
    assert st.read(s).code == 0 and want[0] == 0
    assert int(cnt.item()) == want[1] == len(sz)
    assert np.array_equal(offs.cpu().numpy().view(np.uint64), want[2])
    assert int(ws[-256:][:4].cpu().numpy().view(np.uint32)[0]) == 1


@pytest.mark.parametrize("maxlen", [252, 1000, 8000])
def test_index_window_sizes(dev, maxlen):
    """Entry windows K = maxlen/4 + 1 across the level-kernel variants
    (64-wide LDS, 16-wide LDS, 16-wide global)."""
    rng = np.random.default_rng(maxlen)
    sizes = list(rng.integers(0, maxlen // 4 + 1, 40000) * 4)
    check_index(_messages(sizes), dev, maxlen)


@pytest.mark.parametrize("name", ["recvar", "rpc", "numerics"])
@pytest.mark.parametrize("seed", range(4))
def test_index_fuzzed_vs_oracle(dev, name, seed):
    """Random byte flips in the marks of a reference message stream: the
    device index stops at the same message with the same error as
    read_message would."""
    n = SMALL_N[name]
    x = golden(name, n, "msgs").copy()
    mo = golden(name, n, "msgoffs", np.uint64)
    rng = np.random.default_rng(seed)
    for _ in range(2):
        i = int(mo[int(rng.integers(0, n))]) + int(rng.integers(0, 4))  # hit a mark byte
        x[i] = np.uint8(rng.integers(0, 256))
    check_index(x, dev, min(plan(name).max_record_bytes, A.INDEX_MAX_MSG))


# ----------------------------------------------------- decode_msgs errors
def _oracle_err(fn):
    try:
        fn()
    except O.OracleError as e:
        return (e.code, e.record, e.op)
    return None


def _gpu_err(fn):
    try:
        fn()
    except M.XdrRuntimeError as e:
        return (e.code, e.record, 0xFFFFFFFF if e.op is None else e.op)
    return None


KERNELS = {"per_lane": (1, 1, 0), "image_window": (3, 2, 0), "specialized": (0, 0, 1)}


@pytest.fixture(params=list(KERNELS))
def forced(request):
    """Plan options forcing one encode and one decode kernel: the plan
    interpreter's, or the plan-specialized ones (codegen.cpp + hiprtc)."""
    enc, dec, spec = KERNELS[request.param]
    return {"var_encode_kernel": enc, "var_decode_kernel": dec, "specialize": spec}


@pytest.mark.parametrize("name", ["recvar", "rpc", "vecrec", "rec128"])
@pytest.mark.parametrize("seed", range(3))
def test_decode_msgs_fuzzed_vs_oracle(dev, forced, name, seed):
    n = SMALL_N[name]
    p = plan(name, **forced)
    mar = M.Marshaler(p, dev)
    x = golden(name, n, "msgs").copy()
    mo = golden(name, n, "msgoffs", np.uint64)
    rng = np.random.default_rng(200 + seed)
    for _ in range(3):
        i = int(rng.integers(0, x.size))
        x[i] = np.uint8(rng.integers(0, 256))
    want = _oracle_err(lambda: O.decode_msgs(p.cp, x, n, mo))
    got = _gpu_err(lambda: mar.decode_msgs(to_dev(x, dev), n, to_dev(mo.view(np.int64), dev)))
    assert got == want


@pytest.mark.parametrize("name", ["recvar", "rpc", "vecrec", "numerics"])
@pytest.mark.parametrize("n", [1, 63, 65, 1000])
def test_msgs_kernels_vs_oracle(dev, forced, name, n):
    p = plan(name, **forced)
    mar = M.Marshaler(p, dev)
    N = SMALL_N[name]
    heap = golden(name, N, "heap")
    nat = golden(name, N, "native")[:n * p.stride]
    want, offs = O.encode_msgs(p.cp, nat, n, heap)
    res = mar.encode_msgs(to_dev(nat, dev), n, to_dev(heap, dev) if heap.size else None)
    assert np.array_equal(res.xdr.cpu().numpy(), want)
    assert np.array_equal(res.offsets.cpu().numpy().view(np.uint64), offs)
    back, bheap = mar.decode_msgs(res.xdr, n, res.offsets)
    o_nat, o_heap = O.decode_msgs(p.cp, want, n, offs)
    assert np.array_equal(back.cpu().numpy(), o_nat)
    if bheap is not None:
        assert np.array_equal(bheap.cpu().numpy(), o_heap)


def test_encode_msgs_capacity(dev, forced):
    p = plan("recvar", **forced)
    mar = M.Marshaler(p, dev)
    n = 300
    nat, heap = W.recvar(n)
    _, offs = O.encode_msgs(p.cp, nat, n, heap)
    for cap in (int(offs[200]) + 2, int(offs[200]) + 10):  # in the mark, then in the record
        want = _oracle_err(lambda: O.encode_msgs(p.cp, nat, n, heap, cap=cap))
        got = _gpu_err(lambda: mar.encode_msgs(to_dev(nat, dev), n, to_dev(heap, dev), capacity=cap))
        assert got == want and want[1] == 200
