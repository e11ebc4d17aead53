"""GPU parity: libxdrgpu.so (through the C ABI) against the reference.

Every comparison is against bytes the REAL reference produced
(tests/golden, made by oracle/ref_golden from xdrpp/marshal.cc) or against
the C restatement oracle where the reference has no fixture (fuzzed error
streams).  XDR is integer work: everything is bit-exact.
"""
import hashlib

import numpy as np
import pytest

from conftest import SMALL_N, golden

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from xdrpp_amd import _abi as A  # noqa: E402
from xdrpp_amd import marshal as M  # noqa: E402
from xdrpp_amd import objects as OB  # noqa: E402
from xdrpp_amd import schemas as S  # noqa: E402
from xdrpp_amd import workloads as W  # noqa: E402
import oracle_bridge as O  # noqa: E402
from xdrpp_amd.xdr_types import compile_plan  # noqa: E402

SCHEMAS = ["numerics", "rec128", "recvar", "rpc", "vecrec", "containertest", "rp_list"]
_plans = {}


def plan(name, **options):
    """The plan of a schema, with launch options (xdrg_plan_set_option)."""
    key = (name, tuple(sorted(options.items())))
    if key not in _plans:
        t = S.numerics_validated if name == "numerics_v" else S.ALL[name]
        _plans[key] = M.Plan(t, options)
    return _plans[key]


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def sha(t):
    return hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()


# ----------------------------------------------------------------- golden
@pytest.mark.parametrize("name", SCHEMAS)
def test_golden_encode(dev, name):
    n = SMALL_N[name]
    p = plan(name)
    mar = M.Marshaler(p, dev)
    nat = golden(name, n, "native")
    heap = golden(name, n, "heap")
    res = mar.encode(to_dev(nat, dev), n, to_dev(heap, dev) if heap.size else None)
    want = golden(name, n, "xdr")
    assert np.array_equal(res.xdr.cpu().numpy(), want)
    if not p.is_fixed:
        offs = golden(name, n, "offsets", np.uint64)
        assert np.array_equal(res.offsets.cpu().numpy().view(np.uint64), offs)


@pytest.mark.parametrize("name", SCHEMAS)
def test_golden_decode(dev, name):
    n = SMALL_N[name]
    p = plan(name)
    mar = M.Marshaler(p, dev)
    x = golden(name, n, "xdr")
    offs = golden(name, n, "offsets", np.uint64)
    t_off = None if p.is_fixed else to_dev(offs.view(np.int64), dev)
    nat, heap = mar.decode(to_dev(x, dev), n, t_off)
    if p.is_fixed:
        assert np.array_equal(nat.cpu().numpy(), golden(name, n, "native"))
    else:
        o_nat, o_heap = O.decode(p.cp, x, n, offs)
        assert np.array_equal(nat.cpu().numpy(), o_nat)
        assert np.array_equal(heap.cpu().numpy(), o_heap)
        # decode -> encode reproduces the reference bytes exactly
        res = mar.encode(nat, n, heap)
        assert np.array_equal(res.xdr.cpu().numpy(), x)


# ------------------------------------------------------------- full size
@pytest.mark.parametrize("name,n", [("rec128", 1 << 20), ("numerics", 1 << 16),
                                    ("recvar", 1 << 16), ("rpc", 1 << 16), ("vecrec", 1 << 16),
                                    ("recvar", 1 << 20), ("rpc", 1 << 20), ("numerics", 1 << 20),
                                    ("vecrec", 1 << 20), ("containertest", 1 << 16), ("containertest", 1 << 20)])
def test_full_size_hash(dev, manifest, name, n):
    h = manifest["hashes"][f"{name}_{n}"]
    p = plan(name)
    mar = M.Marshaler(p, dev)
    nat, heap = W.GENERATORS[name](n)
    assert hashlib.sha256(nat.tobytes()).hexdigest() == h["native"]
    t_nat = to_dev(nat, dev)
    t_heap = to_dev(heap, dev) if heap.size else None
    res = mar.encode(t_nat, n, t_heap)
    assert res.xdr.numel() == h["xdr_bytes"]
    assert sha(res.xdr) == h["xdr"]
    back, bheap = mar.decode(res.xdr, n, res.offsets)
    if p.is_fixed:
        assert torch.equal(back, t_nat)
    else:
        assert sha(res.offsets) == h["offsets"]
        res2 = mar.encode(back, n, bheap)
        assert torch.equal(res2.xdr, res.xdr)  # round trip is the identity on the wire


def test_config5_16m_sharded(dev, manifest):
    """BASELINE.json config 5 on one GPU: 16M rec128 records (seed
    0x5EED0005 over the global record index), generated as the 8 shards of
    2M records bench.py gives 8 ranks.  Encoding the shards one by one into
    their slices of one stream (what 8 GPUs + the gather produce) and
    encoding the whole batch in one launch both give the reference's bytes
    (sha256 of xdr_to_opaque over all 16M records); decode round-trips."""
    from xdrpp_amd import shard as SH
    h = manifest["hashes"]["rec128_mgpu_16777216"]
    world, per = 8, 1 << 21
    p = plan("rec128")
    mar = M.Marshaler(p, dev)
    W_ = p.fixed_size
    nat = torch.empty(world * per * p.stride, dtype=torch.uint8, device=dev)
    hn = hashlib.sha256()
    for r in range(world):
        shard, _ = SH.shard_inputs("rec128", per, r, world)
        hn.update(shard.tobytes())
        nat[r * per * p.stride:(r + 1) * per * p.stride] = to_dev(shard, dev)
    assert hn.hexdigest() == h["native"]
    out = torch.empty(world * per * W_, dtype=torch.uint8, device=dev)
    for r in range(world):
        mar.status.init(M._stream())
        mar.launch_encode(nat[r * per * p.stride:(r + 1) * per * p.stride], per,
                          out[r * per * W_:(r + 1) * per * W_])
        mar.check()
    assert sha(out) == h["xdr"]
    whole = mar.encode(nat, world * per)
    assert torch.equal(whole.xdr, out)
    del whole
    back, _ = mar.decode(out, world * per)
    assert torch.equal(back, nat)


# -------------------------------------------------------------- KAT
def test_known_answers(dev, kat):
    mar = M.Marshaler(plan("numerics"), dev)
    nat, _ = W.numerics(1)
    assert mar.encode(to_dev(nat, dev), 1).xdr.cpu().numpy().tobytes().hex() == kat["numerics_marshal_cc"]
    mar = M.Marshaler(plan("rec128"), dev)
    nat, _ = W.rec128(1)
    assert mar.encode(to_dev(nat, dev), 1).xdr.cpu().numpy().tobytes().hex() == kat["rec128_0"]
    mar = M.Marshaler(plan("rpc"), dev)
    nat, heap = W.rpc(64)
    res = mar.encode(to_dev(nat, dev), 64, to_dev(heap, dev))
    offs = res.offsets.cpu().numpy()
    x = res.xdr.cpu().numpy()
    for i, want in enumerate(kat["rpc_first64"]):
        assert x[offs[i]:offs[i + 1]].tobytes().hex() == want


def _recvar_record(bl):
    """recvar with lengths as in ref_golden kat(): blob 1..bl, name 'h'*((3bl)%7)."""
    t = S.recvar
    buf = np.zeros(t.size, dtype=np.uint8)
    heap = bytes(range(1, bl + 1)) + b"h" * ((bl * 3) % 7)

    def put(off, v, dt):
        buf[off:off + np.dtype(dt).itemsize] = np.array([v], dtype=dt).view(np.uint8)
    put(t.offsets["id"], 0x0102030405060708, "<u8")
    put(t.offsets["kind"], -2, "<i4")
    put(t.offsets["blob"], 0, "<u8")
    put(t.offsets["blob"] + 8, bl, "<u4")
    put(t.offsets["name"], bl, "<u8")
    put(t.offsets["name"] + 8, (bl * 3) % 7, "<u4")
    put(t.offsets["score"], 1.5, "<f8")
    return buf, np.frombuffer(heap, dtype=np.uint8).copy()


@pytest.mark.parametrize("bl", range(8))
def test_recvar_residues(dev, kat, bl):
    mar = M.Marshaler(plan("recvar"), dev)
    nat, heap = _recvar_record(bl)
    res = mar.encode(to_dev(nat, dev), 1, to_dev(heap, dev) if heap.size else None)
    assert res.xdr.cpu().numpy().tobytes().hex() == kat[f"recvar_len{bl}"]


# ------------------------------------------------------------ error cases
EXC_NAME = {"xdr_overflow": M.XdrOverflow, "xdr_stack_overflow": M.XdrStackOverflow,
            "xdr_bad_message_size": M.XdrBadMessageSize,
            "xdr_bad_discriminant": M.XdrBadDiscriminant,
            "xdr_should_be_zero": M.XdrShouldBeZero,
            "xdr_invariant_failed": M.XdrInvariantFailed}


@pytest.mark.parametrize("case", [
    "numerics_ok", "numerics_short", "numerics_trailing", "numerics_not_mult4",
    "numerics_bool2", "numerics_enum99_novalidate", "numerics_enum99_validate",
    "recvar_ok", "recvar_nonzero_pad", "recvar_blob_over_bound", "recvar_name_over_bound",
    "recvar_len_past_end", "rpc_ok", "rpc_bad_mtype", "rpc_denied_ok", "rpc_bad_reject_stat",
    "rpc_bad_reply_stat", "vecrec_ok", "vecrec_vals_over_bound", "vecrec_pointer_two",
    "vecrec_pairs_past_end", "vecrec_bool2"])
def test_reference_error_cases(dev, kat, case):
    """Decode the reference's error inputs; exception class and what() must
    equal what the reference threw (tests/golden/kat.json)."""
    c = kat["errors"][case]
    schema = case.split("_")[0]
    pname = "numerics_v" if case == "numerics_enum99_validate" else schema
    p = plan(pname)
    mar = M.Marshaler(p, dev)
    x = np.frombuffer(bytes.fromhex(c["input"]), dtype=np.uint8).copy()
    offs = None
    if not p.is_fixed:
        offs = to_dev(np.array([0, x.size], dtype=np.int64), dev)
    t_x = to_dev(x, dev) if x.size else torch.empty(0, dtype=torch.uint8, device=dev)
    if c["exception"] == "none":
        nat, _ = mar.decode(t_x, 1, offs)
        if case == "numerics_bool2":
            assert nat.cpu().numpy()[0] == 1  # any nonzero decodes as true
        return
    with pytest.raises(EXC_NAME[c["exception"]]) as ei:
        mar.decode(t_x, 1, offs)
    assert str(ei.value) == c["what"]
    # trailing bytes after the last record are reported past it (record n)
    assert ei.value.record == (1 if case == "numerics_trailing" else 0)


# --------------------------------------------- batch errors vs the oracle
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


@pytest.mark.parametrize("name", ["numerics_v", "recvar", "rpc", "vecrec"])
@pytest.mark.parametrize("seed", range(6))
def test_fuzzed_stream_errors_match_oracle(dev, name, seed):
    """Flip random bytes of a valid batch stream; the first failing record,
    its op and the error code must match the C restatement, and every
    record before it must decode identically."""
    base = "numerics" if name == "numerics_v" else name
    n = SMALL_N[base]
    p = plan(name)
    mar = M.Marshaler(p, dev)
    x = golden(base, n, "xdr").copy()
    offs = golden(base, n, "offsets", np.uint64)
    rng = np.random.default_rng(seed)
    for _ in range(3):
        i = int(rng.integers(0, x.size))
        x[i] = np.uint8(rng.integers(0, 256))
    o_off = None if p.is_fixed else offs
    want = _oracle_err(lambda: O.decode(p.cp, x, n, o_off))
    t_off = None if p.is_fixed else to_dev(offs.view(np.int64), dev)
    got = _gpu_err(lambda: mar.decode(to_dev(x, dev), n, t_off))
    assert got == want


@pytest.mark.parametrize("n", [0, 1, 3, 255, 257, 1023])
@pytest.mark.parametrize("name", SCHEMAS)
def test_ragged_batch_sizes(dev, name, n):
    p = plan(name)
    mar = M.Marshaler(p, dev)
    nat, heap = W.GENERATORS[name](max(n, 1))
    nat = nat[:n * p.stride]
    want, offs = O.encode(p.cp, nat, n, heap)
    t_nat = to_dev(nat, dev) if n else torch.empty(0, dtype=torch.uint8, device=dev)
    res = mar.encode(t_nat, n, to_dev(heap, dev) if heap.size else None)
    assert np.array_equal(res.xdr.cpu().numpy(), want)
    back, bheap = mar.decode(res.xdr, n, res.offsets)
    o_nat, o_heap = O.decode(p.cp, want, n, None if p.is_fixed else offs)
    assert np.array_equal(back.cpu().numpy(), o_nat)


@pytest.mark.parametrize("name", ["numerics", "rec128"])
def test_unaligned_buffers(dev, name):
    """4-byte-aligned (not 16) device buffers take the scalar-load variant."""
    n = 333
    p = plan(name)
    mar = M.Marshaler(p, dev)
    nat, _ = W.GENERATORS[name](n)
    big = torch.zeros(nat.size + 16, dtype=torch.uint8, device=dev)
    big[4:4 + nat.size] = to_dev(nat, dev)
    src = big[4:4 + nat.size]
    out = torch.zeros(n * p.fixed_size + 16, dtype=torch.uint8, device=dev)[4:4 + n * p.fixed_size]
    s = torch.cuda.current_stream().cuda_stream
    mar.status.init(s)
    mar.launch_encode(src, n, out)
    mar.check()
    want, _ = O.encode(p.cp, nat, n)
    assert np.array_equal(out.cpu().numpy(), want)


def test_fixed_capacity_and_length_errors(dev):
    p = plan("numerics")
    mar = M.Marshaler(p, dev)
    n = 100
    nat, _ = W.numerics(n)
    t_nat = to_dev(nat, dev)
    cap = 44 * 37 + 16  # record 37 runs out at op 3 (i3 needs bytes 12..20)
    with pytest.raises(M.XdrOverflow) as ei:
        mar.encode(t_nat, n, capacity=cap)
    assert str(ei.value) == "insufficient buffer space in xdr_generic_put"
    assert (ei.value.record, ei.value.op) == (37, 3)
    assert _oracle_err(lambda: O.encode(p.cp, nat, n, cap=cap)) == (A.ERR_OVERFLOW_PUT, 37, 3)
    x = golden("numerics", 1000, "xdr")[:44 * 100]
    for L, exc, rec in ((44 * 50 + 8, M.XdrOverflow, 50), (44 * 100 + 4, M.XdrBadMessageSize, 100),
                        (44 * 100 - 2, M.XdrBadMessageSize, 0)):
        xx = np.zeros(L, dtype=np.uint8)
        xx[:min(L, x.size)] = x[:min(L, x.size)]
        with pytest.raises(exc) as ei:
            mar.decode(to_dev(xx, dev), n)
        assert ei.value.record == rec
        want = _oracle_err(lambda: O.decode(p.cp, xx, n))
        assert (ei.value.code, ei.value.record) == want[:2]


@pytest.mark.parametrize("name,limit", [("numerics", 0), ("numerics", 1), ("rpc", 3),
                                        ("rpc", 4), ("rpc", 5), ("recvar", 0)])
def test_stack_limit(dev, name, limit):
    """marshaling_stack_limit (marshal.h:21,34,131-136,198-205)."""
    n = 64
    p = plan(name)
    mar = M.Marshaler(p, dev)
    nat, heap = W.GENERATORS[name](n)
    t_heap = to_dev(heap, dev) if heap.size else None
    want = _oracle_err(lambda: O.encode(p.cp, nat, n, heap, stack_limit=limit))
    got = _gpu_err(lambda: mar.encode(to_dev(nat, dev), n, t_heap, stack_limit=limit))
    assert got == want
    x, offs = O.encode(p.cp, nat, n, heap)
    o_off = None if p.is_fixed else offs
    t_off = None if p.is_fixed else to_dev(offs.view(np.int64), dev)
    want = _oracle_err(lambda: O.decode(p.cp, x, n, o_off, stack_limit=limit))
    got = _gpu_err(lambda: mar.decode(to_dev(x, dev), n, t_off, stack_limit=limit))
    assert got == want


def test_bad_discriminant_encode(dev):
    p = plan("rpc")
    mar = M.Marshaler(p, dev)
    n = 200
    nat, heap = W.rpc(n)
    nat = nat.reshape(n, p.stride).copy()
    mt = S.rpc_msg.offset_of("body")
    nat[150, mt:mt + 4] = np.array([7], dtype="<u4").view(np.uint8)
    nat[170, mt:mt + 4] = np.array([9], dtype="<u4").view(np.uint8)
    nat = nat.reshape(-1)
    with pytest.raises(M.XdrBadDiscriminant) as ei:
        mar.encode(to_dev(nat, dev), n, to_dev(heap, dev))
    assert str(ei.value) == "bad value of mtype in _body_t"
    assert ei.value.record == 150
    assert _oracle_err(lambda: O.encode(p.cp, nat, n, heap))[:2] == (A.ERR_BAD_DISCRIMINANT, 150)


def test_swaps(dev):
    x = np.random.default_rng(1).integers(0, 2**63, 100003, dtype=np.int64)
    t = to_dev(x, dev)
    assert np.array_equal(M.swap64(t).cpu().numpy(), x.byteswap())
    x32 = x.view(np.int32)
    assert np.array_equal(M.swap32(to_dev(x32, dev)).cpu().numpy(), x32.byteswap())


# ------------------------------------- every var kernel, forced in turn
# (encode kernel, decode kernel, specialize, stage_bytes): the window decode
# of plans with fixed-element containers (vecrec) stages a group's element
# arrays in LDS when they fit (-1: the default 8 KiB), writes them straight
# from the walk otherwise (0: never staged; 1024: some groups staged, some not)
KERNELS = {"per_lane": (1, 1, 0, -1), "chunk_image_window": (3, 2, 0, -1), "window_mixed_stage": (3, 2, 0, 1024),
           "specialized": (0, 0, 1, -1), "specialized_no_stage": (0, 0, 1, 0),
           "specialized_mixed_stage": (0, 0, 1, 1024)}


@pytest.fixture(params=list(KERNELS))
def forced(request):
    """Plan options forcing one encode and one decode kernel: the plan
    interpreter's, or the plan-specialized ones (codegen.cpp + hiprtc)."""
    enc, dec, spec, stage = KERNELS[request.param]
    return {"var_encode_kernel": enc, "var_decode_kernel": dec, "specialize": spec, "stage_bytes": stage}


@pytest.mark.parametrize("name", ["recvar", "rpc", "vecrec"])
@pytest.mark.parametrize("n", [1, 63, 65, 1024])
def test_var_kernels_golden(dev, forced, name, n):
    p = plan(name, **forced)
    mar = M.Marshaler(p, dev)
    N = SMALL_N[name]
    nat_all = golden(name, N, "native")
    heap = golden(name, N, "heap")
    nat = nat_all[:n * p.stride]
    want, offs = O.encode(p.cp, nat, n, heap)
    res = mar.encode(to_dev(nat, dev), n, to_dev(heap, dev))
    assert np.array_equal(res.xdr.cpu().numpy(), want)
    assert np.array_equal(res.offsets.cpu().numpy().view(np.uint64), offs)
    back, bheap = mar.decode(res.xdr, n, res.offsets)
    o_nat, o_heap = O.decode(p.cp, want, n, offs)
    assert np.array_equal(back.cpu().numpy(), o_nat)
    assert np.array_equal(bheap.cpu().numpy(), o_heap)


@pytest.mark.parametrize("name", ["recvar", "rpc", "vecrec"])
@pytest.mark.parametrize("seed", range(3))
def test_var_kernels_fuzzed_errors(dev, forced, name, seed):
    n = SMALL_N[name]
    p = plan(name, **forced)
    mar = M.Marshaler(p, dev)
    x = golden(name, n, "xdr").copy()
    offs = golden(name, n, "offsets", np.uint64)
    rng = np.random.default_rng(100 + seed)
    for _ in range(3):
        i = int(rng.integers(0, x.size))
        x[i] = np.uint8(rng.integers(0, 256))
    want = _oracle_err(lambda: O.decode(p.cp, x, n, offs))
    got = _gpu_err(lambda: mar.decode(to_dev(x, dev), n, to_dev(offs.view(np.int64), dev)))
    assert got == want


@pytest.mark.parametrize("bad", ["reversed", "past_end"])
def test_var_kernels_bad_offsets(dev, forced, bad):
    """Offsets the decode refuses (record 70: b < a, or b past the stream)
    inside a group of packed element arrays: the oracle's error, the records
    before it decoded identically, nothing written past the heap."""
    n = 200
    p = plan("vecrec", **forced)
    mar = M.Marshaler(p, dev)
    nat, heap = W.GENERATORS["vecrec"](n)
    x, offs = O.encode(p.cp, nat, n, heap)
    offs = offs.copy()
    offs[71] = offs[70] - 8 if bad == "reversed" else x.size + 64
    want = _oracle_err(lambda: O.decode(p.cp, x, n, offs))
    assert want[:2] == (A.ERR_OVERFLOW_GET, 70)
    H = p.decode_heap_bytes(x.size)
    guard = 4096
    hout = torch.full((H + guard,), 0xA5, dtype=torch.uint8, device=dev)
    back = torch.zeros(n * p.stride, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    mar.status.init(s)
    mar.launch_decode(to_dev(x, dev), n, back, offsets=to_dev(offs.view(np.int64), dev), heap_out=hout[:H],
                      stream=s)
    assert _gpu_err(lambda: mar.check(s)) == want
    assert bool((hout[H:] == 0xA5).all()), "decode wrote past its heap"
    # records 0..69 hold what the oracle decodes from them alone (values:
    # the element arrays' places depend on the batch's length)
    o_nat, o_heap = O.decode(p.cp, x[:int(offs[70])], 70, offs[:71])
    t = S.ALL["vecrec"]
    assert OB.unstage(t, back.cpu().numpy()[:70 * p.stride], hout[:H].cpu().numpy(), 70) == \
        OB.unstage(t, o_nat, o_heap, 70)


@pytest.mark.parametrize("name", ["recvar", "rpc", "vecrec"])
def test_var_kernels_capacity_and_stack(dev, forced, name):
    n = 300
    p = plan(name, **forced)
    mar = M.Marshaler(p, dev)
    nat, heap = W.GENERATORS[name](n)
    full, offs = O.encode(p.cp, nat, n, heap)
    cap = int(offs[200]) + 10  # record 200 runs out of room
    want = _oracle_err(lambda: O.encode(p.cp, nat, n, heap, cap=cap))
    got = _gpu_err(lambda: mar.encode(to_dev(nat, dev), n, to_dev(heap, dev), capacity=cap))
    assert got == want and want[1] == 200
    for limit in (0, 1, 3):
        want = _oracle_err(lambda: O.encode(p.cp, nat, n, heap, stack_limit=limit))
        got = _gpu_err(lambda: mar.encode(to_dev(nat, dev), n, to_dev(heap, dev), stack_limit=limit))
        assert got == want


# ------------------------------------------------------------ depth_checker
@pytest.mark.parametrize("name", SCHEMAS)
def test_record_depths_golden(dev, name):
    """xdrg_record_depths vs the real check_xdr_depth (xdrpp/depth_checker.h):
    depths[i] is the smallest limit record i passes, so check_xdr_depth(r, L)
    == depths <= L at every L."""
    n = SMALL_N[name]
    mar = M.Marshaler(plan(name), dev)
    nat = to_dev(golden(name, n, "native"), dev)
    hp = golden(name, n, "heap")
    heap = to_dev(hp, dev) if hp.size else None  # element arrays of subroutine containers
    want = golden(name, n, "depths", np.uint32)
    got = mar.record_depths(nat, n, heap).cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want)
    for lim in range(int(want.max()) + 2):
        assert np.array_equal(mar.check_xdr_depth(nat, n, lim, heap).cpu().numpy(), want <= lim)


@pytest.mark.parametrize("name,n", [("rpc", 1 << 20), ("vecrec", 1 << 16)])
def test_record_depths_full_size(dev, name, n):
    p = plan(name)
    nat, _ = W.GENERATORS[name](n)
    got = M.Marshaler(p, dev).record_depths(to_dev(nat, dev), n).cpu().numpy().view(np.uint32)
    assert np.array_equal(got, O.depths(p.cp, nat, n))


# ------------------------------------- fixed non-identity paths (group / LDS)
FIXED_PATHS = {"auto": 0, "lds": 2}
BOOLS = S.Struct("boolrec", [("a", S.Bool), ("b", S.Bool), ("c", S.Int), ("d", S.Bool)])


@pytest.fixture(params=list(FIXED_PATHS))
def fixed_path(request):
    return {"fixed_path": FIXED_PATHS[request.param]}


@pytest.mark.parametrize("n", [1, 3, 4, 5, 1000, 4099, 1 << 16])
def test_fixed_group_numerics(dev, fixed_path, n):
    """numerics (56-byte native, 44-byte wire): full groups of 4 records on
    the group kernel, the tail on the LDS kernel; both paths bit-exact."""
    p = plan("numerics", **fixed_path)
    nat, _ = W.numerics(n)
    want, _ = O.encode(p.cp, nat, n)
    mar = M.Marshaler(p, dev)
    res = mar.encode(to_dev(nat, dev), n)
    assert np.array_equal(res.xdr.cpu().numpy(), want)
    back, _ = mar.decode(res.xdr, n)
    assert np.array_equal(back.cpu().numpy(), nat)


@pytest.mark.parametrize("n", [1, 4, 7, 4096, 10001])
def test_fixed_group_bools(dev, fixed_path, n):
    """Several bools per native word (decode: 2 terms per word) and a bool
    in the record's last word (encode: the window's high word)."""
    cp = compile_plan(BOOLS)
    p = M.Plan(BOOLS, fixed_path)
    rng = np.random.default_rng(n)
    nat = rng.integers(0, 256, size=n * cp.stride, dtype=np.uint8)
    want, _ = O.encode(cp, nat, n)
    mar = M.Marshaler(p, dev)
    res = mar.encode(to_dev(nat, dev), n)
    assert np.array_equal(res.xdr.cpu().numpy(), want)
    # decode arbitrary nonzero wire bools (xdr_traits<bool>: nonzero is true)
    wire = want.view("<u4").copy().reshape(n, 4)
    wire[:, [0, 1, 3]] = rng.integers(0, 3, size=(n, 3)).astype(">u4").view("<u4")
    wire = wire.reshape(-1).view(np.uint8)
    o_nat, _ = O.decode(cp, wire, n, None)
    back, _ = mar.decode(to_dev(wire, dev), n)
    assert np.array_equal(back.cpu().numpy(), o_nat)


# ----------------------- chunk-map encode: LDS image sizes and unroll depths
@pytest.fixture(params=[(-1, 8), (0, 8), (1024, 4), (4096, 16)], ids=lambda v: f"img{v[0]}_u{v[1]}")
def enc_shape(request):
    return {"image_bytes": request.param[0], "enc_unroll": request.param[1]}


@pytest.mark.parametrize("name", ["recvar", "rpc", "vecrec"])
@pytest.mark.parametrize("n", [1, 64, 1000, 4099])
def test_encode_image_shapes(dev, enc_shape, name, n):
    """Every stretch byte goes through the LDS image or the direct global
    path (whole 16-byte chunks as one store); both, at every image size and
    unroll depth, give the reference's bytes."""
    p = plan(name, **enc_shape)
    nat, heap = W.GENERATORS[name](n)
    want, offs = O.encode(p.cp, nat, n, heap)
    res = M.Marshaler(p, dev).encode(to_dev(nat, dev), n, to_dev(heap, dev) if heap.size else None)
    assert np.array_equal(res.xdr.cpu().numpy(), want)
    assert np.array_equal(res.offsets.cpu().numpy().view(np.uint64), offs)


@pytest.fixture(params=[(-1, 1), (2048, 0), (16384, 1)], ids=lambda v: f"win{v[0]}_ra{v[1]}")
def dec_shape(request):
    return {"window_bytes": request.param[0], "dec_readahead": request.param[1]}


@pytest.mark.parametrize("name", ["recvar", "rpc", "vecrec"])
@pytest.mark.parametrize("n", [1, 64, 1000, 4099])
def test_decode_window_shapes(dev, dec_shape, name, n):
    """Stream words inside the LDS window, past it through the 32-byte
    read-ahead, or past it word by word: the same records as the C
    restatement."""
    p = plan(name, **dec_shape)
    nat, heap = W.GENERATORS[name](n)
    want, offs = O.encode(p.cp, nat, n, heap)
    back, bheap = M.Marshaler(p, dev).decode(to_dev(want, dev), n, to_dev(offs.view(np.int64), dev))
    o_nat, o_heap = O.decode(p.cp, want, n, offs)
    assert np.array_equal(back.cpu().numpy(), o_nat)
    assert np.array_equal(bheap.cpu().numpy(), o_heap)


@pytest.mark.parametrize("linear", [1, 0, -1])
@pytest.mark.parametrize("n", [1, 63, 65, 300, 4099])
def test_size_pass_linear(dev, linear, n):
    """recvar is a linear plan (no unions/containers): its size pass reads
    the length words without a walk; both passes give xdr_size and the
    same encode."""
    p = plan("recvar", size_linear=linear)
    nat, heap = W.recvar(n)
    want, offs = O.encode(p.cp, nat, n, heap)
    mar = M.Marshaler(p, dev)
    sz = mar.serial_sizes(to_dev(nat, dev), n).cpu().numpy().astype(np.uint64)
    assert np.array_equal(sz, np.diff(offs))
    res = mar.encode(to_dev(nat, dev), n, to_dev(heap, dev))
    assert np.array_equal(res.xdr.cpu().numpy(), want)
    msgs = mar.encode_msgs(to_dev(nat, dev), n, to_dev(heap, dev))
    assert np.array_equal(msgs.xdr.cpu().numpy(), O.encode_msgs(p.cp, nat, n, heap)[0])


@pytest.mark.parametrize("name", ["recvar", "rpc", "vecrec"])
@pytest.mark.parametrize("n", [64, 65, 4099, 100003])
def test_encode_sizes_scan_index(dev, name, n):
    """Size pass + block scan + encode: the reference's bytes, record index
    and total, for batches that end inside a 64-record block and span
    several scan tiles."""
    p = plan(name)
    nat, heap = W.GENERATORS[name](n)
    want, offs = O.encode(p.cp, nat, n, heap)
    mar = M.Marshaler(p, dev)
    res = mar.encode(to_dev(nat, dev), n, to_dev(heap, dev) if heap.size else None)
    assert np.array_equal(res.xdr.cpu().numpy(), want)
    assert np.array_equal(res.offsets.cpu().numpy().view(np.uint64), offs)
    m = mar.encode_msgs(to_dev(nat, dev), n, to_dev(heap, dev) if heap.size else None)
    assert np.array_equal(m.xdr.cpu().numpy(), O.encode_msgs(p.cp, nat, n, heap)[0])


def test_encode_bad_discriminant_lowest_record(dev):
    """A bad discriminant found by the size pass is reported at the lowest
    failing record, with the reference's what()."""
    p = plan("rpc")
    n = 5000
    nat, heap = W.rpc(n)
    rec = nat.reshape(n, p.stride).copy()
    off = S.rpc_msg.offset_of("body")
    for bad in (4321, 777):
        rec[bad, off:off + 4] = np.frombuffer(np.uint32(9).tobytes(), np.uint8)
    with pytest.raises(M.XdrBadDiscriminant) as ei:
        M.Marshaler(p, dev).encode(to_dev(rec.reshape(-1), dev), n, to_dev(heap, dev))
    assert ei.value.record == 777
    assert str(ei.value) == "bad value of mtype in _body_t"


# ------------------------------------------------- vector element layouts
# Element structs that take the register-staged element path (<= 16 bytes of
# word-aligned scalars and bools, bools sharing a word, 12-byte strides) and
# ones that take the per-field path (an opaque field, > 16 bytes).
_e_opq = S.Struct("e_opq", [("a", S.Int), ("t", S.OpaqueArray(3)), ("f", S.Bool)])
_e_wide = S.Struct("e_wide", [("a", S.Hyper), ("b", S.Hyper), ("c", S.UInt)])
_e_bools = S.Struct("e_bools", [("a", S.Bool), ("b", S.Bool), ("c", S.Int)])
_e_three = S.Struct("e_three", [("a", S.Int), ("b", S.UInt), ("c", S.Int)])
_e_ih = S.Struct("e_ih", [("a", S.Int), ("b", S.Hyper)])
vshapes = S.Struct("vshapes", [("v1", S.XVector(_e_opq, 5)), ("v2", S.XVector(_e_wide, 3)),
                               ("v3", S.XVector(_e_bools, 4)), ("v4", S.XVector(_e_three, 6)),
                               ("v5", S.XVector(_e_ih, 3)), ("v6", S.XVector(S.Hyper, 4)),
                               ("tail", S.UInt)])
_VS = [("v1", _e_opq, 5), ("v2", _e_wide, 3), ("v3", _e_bools, 4), ("v4", _e_three, 6),
       ("v5", _e_ih, 3), ("v6", S.Hyper, 4)]


def _vshapes_batch(n, seed, straddle=False):
    """Random records; element bytes random (bools included), arrays 8-byte
    aligned in the heap.  With `straddle` the last record's v4 array starts
    5 bytes before the end of the heap, so its elements are read past it."""
    rng = np.random.default_rng(seed)
    o = vshapes.offsets
    nat = np.zeros((n, vshapes.size), dtype=np.uint8)
    heap = bytearray()
    for r in range(n):
        for f, et, mx in _VS:
            cnt = int(rng.integers(0, mx + 1))
            start = len(heap)
            heap += rng.integers(0, 256, cnt * et.size, dtype=np.uint8).tobytes()
            heap += bytes(-len(heap) % 8)
            _ref(nat, r, o[f], start, cnt)
        nat[r, o["tail"]:o["tail"] + 4] = rng.integers(0, 256, 4, dtype=np.uint8)
    if straddle:
        heap += rng.integers(0, 256, 8, dtype=np.uint8).tobytes()
        _ref(nat, n - 1, o["v4"], len(heap) - 5, 2)
    return nat.reshape(-1), np.frombuffer(bytes(heap), np.uint8).copy()


def _ref(nat, r, off, start, cnt):
    nat[r, off:off + 8] = np.frombuffer(np.uint64(start).tobytes(), np.uint8)
    nat[r, off + 8:off + 12] = np.frombuffer(np.uint32(cnt).tobytes(), np.uint8)


@pytest.mark.parametrize("straddle", [False, True])
@pytest.mark.parametrize("n", [1, 64, 257])
def test_vector_element_layouts(dev, forced, n, straddle):
    p = M.Plan(vshapes, forced)
    mar = M.Marshaler(p, dev)
    nat, heap = _vshapes_batch(n, 900 + n, straddle)
    # the oracle reads the heap unclamped: give it the zeros the GPU reads
    # past heap_len
    want, offs = O.encode(p.cp, nat, n, np.concatenate([heap, np.zeros(64, np.uint8)]))
    res = mar.encode(to_dev(nat, dev), n, to_dev(heap, dev))
    assert np.array_equal(res.xdr.cpu().numpy(), want)
    assert np.array_equal(res.offsets.cpu().numpy().view(np.uint64), offs)
    back, bheap = mar.decode(res.xdr, n, res.offsets)
    o_nat, o_heap = O.decode(p.cp, want, n, offs)
    assert np.array_equal(back.cpu().numpy(), o_nat)
    assert np.array_equal(bheap.cpu().numpy(), o_heap)
