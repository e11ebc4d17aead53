"""CPU: the oracle and the workload generators against the reference.

The fixtures in tests/golden were produced by the REAL reference
(xdrpp/marshal.cc compiled in place by oracle/Makefile into
oracle/_ref/ref_golden, script oracle/make_golden.py).  These tests pin:

  * the C restatement oracle (oracle/xdr_oracle.c) -- encode, decode, the
    error cases and their ordering -- to the reference's bytes and
    exceptions, so that it can stand in as the checker for inputs the
    fixtures do not cover (fuzzed error streams in the GPU tests);
  * the numpy generators (xdrpp_amd/workloads.py) to the reference-side
    generator (oracle/workload_gen.h), byte for byte, at fixture size and
    through the manifest's sha256 at full size;
  * the host-side error mapping (exception class + what(), marshal.error_from)
    to the reference's exceptions (kat.json "errors").

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

SCHEMAS = ["numerics", "rec128", "recvar", "rpc", "vecrec", "containertest", "rp_list"]
CP = {k: compile_plan(t) for k, t in S.ALL.items()}
CP["numerics_v"] = compile_plan(S.numerics_validated)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# ----------------------------------------------------------- generators
@pytest.mark.parametrize("name", SCHEMAS)
def test_generator_matches_reference_fixture(name):
    n = SMALL_N[name]
    nat, heap = W.GENERATORS[name](n)
    assert np.array_equal(nat, golden(name, n, "native"))
    assert np.array_equal(heap, golden(name, n, "heap"))


@pytest.mark.parametrize("key", ["numerics_65536", "recvar_65536", "rpc_65536", "vecrec_65536",
                                 "containertest_65536", "rp_list_65536", "rec128_1048576"])
def test_generator_matches_manifest(manifest, key):
    name, n = key.rsplit("_", 1)
    h = manifest["hashes"][key]
    nat, heap = W.GENERATORS[name](int(n))
    assert sha(nat) == h["native"]
    assert sha(heap) == h["heap"]


@pytest.mark.parametrize("name", SCHEMAS)
def test_generator_first_is_a_slice(name):
    """Shard generation (first=k) reproduces records [k, k+n) of the batch."""
    nat, heap = W.GENERATORS[name](96)
    sub, sheap = W.GENERATORS[name](32, first=64)
    stride = CP[name].stride
    assert len(sub) == 32 * stride
    if not heap.size:
        assert np.array_equal(sub, nat[64 * stride:])
    else:
        # same encodings (heap offsets are shard-local)
        whole, woffs = O.encode(CP[name], nat, 96, heap)
        part, _ = O.encode(CP[name], sub, 32, sheap)
        assert np.array_equal(part, whole[int(woffs[64]):])


# ------------------------------------------------------- oracle encode
@pytest.mark.parametrize("name", SCHEMAS)
def test_oracle_encode_golden(name):
    n = SMALL_N[name]
    heap = golden(name, n, "heap")
    x, offs = O.encode(CP[name], golden(name, n, "native"), n, heap)
    assert np.array_equal(x, golden(name, n, "xdr"))
    assert np.array_equal(offs, golden(name, n, "offsets", np.uint64))


@pytest.mark.parametrize("name", SCHEMAS)
def test_oracle_decode_golden(name):
    n = SMALL_N[name]
    x = golden(name, n, "xdr")
    offs = golden(name, n, "offsets", np.uint64)
    nat, heap = O.decode(CP[name], x, n, offs)
    if not CP[name].is_var:
        assert np.array_equal(nat, golden(name, n, "native"))
    else:
        # the decoded batch has its own heap layout; it must encode back to
        # the reference's bytes
        x2, offs2 = O.encode(CP[name], nat, n, heap)
        assert np.array_equal(x2, x)
        assert np.array_equal(offs2, offs)


@pytest.mark.parametrize("key", ["numerics_65536", "recvar_65536", "rpc_65536", "vecrec_65536",
                                 "containertest_65536", "rp_list_65536", "rec128_1048576"])
def test_oracle_full_size_hash(manifest, key):
    name, n = key.rsplit("_", 1)
    n = int(n)
    h = manifest["hashes"][key]
    nat, heap = W.GENERATORS[name](n)
    x, offs = O.encode(CP[name], nat, n, heap)
    assert x.size == h["xdr_bytes"]
    assert sha(x) == h["xdr"]
    if CP[name].is_var:
        assert sha(offs) == h["offsets"]


# --------------------------------------------------------------- KATs
def test_oracle_known_answers(kat):
    nat, _ = W.numerics(1)
    assert O.encode(CP["numerics"], nat, 1)[0].tobytes().hex() == kat["numerics_marshal_cc"]
    nat, _ = W.rec128(1)
    assert O.encode(CP["rec128"], nat, 1)[0].tobytes().hex() == kat["rec128_0"]
    nat, heap = W.rpc(64)
    x, offs = O.encode(CP["rpc"], nat, 64, heap)
    for i, want in enumerate(kat["rpc_first64"]):
        assert x[offs[i]:offs[i + 1]].tobytes().hex() == want


@pytest.mark.parametrize("bl", range(8))
def test_oracle_recvar_residues(kat, bl):
    """Payload lengths 0..7 (every pad residue), reference bytes."""
    t = S.recvar
    buf = np.zeros(t.size, dtype=np.uint8)
    heap = np.frombuffer(bytes(range(1, bl + 1)) + b"h" * ((bl * 3) % 7), dtype=np.uint8).copy()

    def put(off, v, dt):
        buf[off:off + np.dtype(dt).itemsize] = np.array([v], dtype=dt).view(np.uint8)
    put(t.offsets["id"], 0x0102030405060708, "<u8")
    put(t.offsets["kind"], -2, "<i4")
    put(t.offsets["blob"], 0, "<u8")
    put(t.offsets["blob"] + 8, bl, "<u4")
    put(t.offsets["name"], bl, "<u8")
    put(t.offsets["name"] + 8, (bl * 3) % 7, "<u4")
    put(t.offsets["score"], 1.5, "<f8")
    assert O.encode(CP["recvar"], buf, 1, heap)[0].tobytes().hex() == kat[f"recvar_len{bl}"]


# ------------------------------------------- reference exceptions (host)
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
def test_oracle_reference_error_cases(kat, case):
    """The oracle's (code, op) for the reference's error inputs, mapped by
    the product's host error path, gives the exception class and what()
    string the reference threw."""
    c = kat["errors"][case]
    schema = case.split("_")[0]
    pname = "numerics_v" if case == "numerics_enum99_validate" else schema
    cp = CP[pname]
    x = np.frombuffer(bytes.fromhex(c["input"]), dtype=np.uint8).copy()
    offs = np.array([0, x.size], dtype=np.uint64) if cp.is_var else None
    try:
        O.decode(cp, x, 1, offs)
        got = None
    except O.OracleError as e:
        got = e
    if c["exception"] == "none":
        assert got is None
        return
    assert got is not None
    plan = M.Plan(cp)  # host-only: plan creation does not touch the device
    err = A.XdrgError(code=got.code, exc=0, record=got.record, op=got.op, rsv=0, total_bytes=0)
    exc = M.error_from(plan, err)
    assert type(exc) is EXC_NAME[c["exception"]]
    assert str(exc) == c["what"]
    assert exc.record == (1 if case == "numerics_trailing" else 0)


def test_oracle_stack_limit():
    """xdr_generic_put/get stack budget (marshal.h:129-136, 192-199): rpc
    nests 6 levels deep; a limit of 5 fails at the first op below it."""
    nat, heap = W.rpc(4)
    with pytest.raises(O.OracleError) as ei:
        O.encode(CP["rpc"], nat, 4, heap, stack_limit=1)
    assert ei.value.code == A.ERR_STACK_PUT and ei.value.record == 0
    x, offs = O.encode(CP["rpc"], nat, 4, heap)
    O.decode(CP["rpc"], x, 4, offs, stack_limit=6)
    with pytest.raises(O.OracleError) as ei:
        O.decode(CP["rpc"], x, 4, offs, stack_limit=1)
    assert ei.value.code == A.ERR_STACK_GET


@pytest.mark.parametrize("name", SCHEMAS)
def test_oracle_depths_golden(name):
    """depth_checker: the C restatement vs the real check_xdr_depth
    (oracle/ref_golden depths: the smallest passing limit per record)."""
    n = SMALL_N[name]
    cp = compile_plan(S.ALL[name])
    d = O.depths(cp, golden(name, n, "native"), n, golden(name, n, "heap"))
    assert np.array_equal(d, golden(name, n, "depths", np.uint32))
