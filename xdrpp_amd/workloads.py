"""Deterministic synthetic record batches for the benchmark configs
(SURVEY.md §8(d)).  numpy restatement of oracle/workload_gen.h +
oracle/ref_golden.cc's generators; tests pin the two together through the
committed fixtures (byte-equal small batches, sha256 of full-size ones).

    draw(seed, i) = splitmix64 finaliser of seed + (i + 1) * GAMMA

Every generator returns (native, heap): ``native`` is n * stride bytes in
the staged layout of the schema (xdrpp_amd.schemas), ``heap`` the payload
bytes the xdrg_bytes_ref fields point into (empty for fixed schemas).
Payload heaps are packed in record order with no alignment, so device
encodes exercise unaligned heap reads.
"""
from __future__ import annotations

import numpy as np

from . import schemas as S

GAMMA = np.uint64(0x9E3779B97F4A7C15)
SEED_NUMERICS = 0x5EED0001
SEED_REC128 = 0x5EED0002
SEED_RECVAR = 0x5EED0003
SEED_RPC = 0x5EED0004
SEED_REC128_MGPU = 0x5EED0005
SEED_VECREC = 0x5EED0006
SEED_CONTAINERTEST = 0x5EED0008
SEED_RP_LIST = 0x5EED0009
RP_LIST_LONG = 500  # nodes of every 65536th list
PAYLOAD_XOR = 0xB10BB10BB10BB10B

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def draw(seed: int, idx: np.ndarray) -> np.ndarray:
    """splitmix64 outputs #idx of the stream seeded with ``seed``."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx.astype(np.uint64) + np.uint64(1)) * GAMMA
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _draws(seed: int, n: int, per: int, first: int = 0) -> np.ndarray:
    idx = (np.arange(first, first + n, dtype=np.uint64)[:, None] * np.uint64(per)
           + np.arange(per, dtype=np.uint64)[None, :])
    return draw(seed, idx)


def _put(buf: np.ndarray, off: int, values: np.ndarray, dt: str) -> None:
    v = np.ascontiguousarray(values.astype(dt))
    k = v.dtype.itemsize
    buf[:, off:off + k] = v.view(np.uint8).reshape(-1, k)


def numerics(n: int, seed: int = SEED_NUMERICS, first: int = 0) -> tuple[np.ndarray, np.ndarray]:
    t = S.numerics
    d = _draws(seed, n, 8, first)
    buf = np.zeros((n, t.size), dtype=np.uint8)
    o = t.offsets
    _put(buf, o["b"], d[:, 0] & np.uint64(1), "u1")
    for f, k, dt in (("i1", 1, "<u4"), ("i2", 2, "<u4"), ("i3", 3, "<u8"), ("i4", 4, "<u8"),
                     ("f1", 5, "<u4"), ("f2", 6, "<u8")):
        _put(buf, o[f], d[:, k] & np.uint64(0xFFFFFFFF) if dt == "<u4" else d[:, k], dt)
    _put(buf, o["e1"], d[:, 7] % np.uint64(3), "<u4")
    if n and first == 0:
        # record 0 = tests/marshal.cc:482-490
        r0 = np.zeros((1, t.size), dtype=np.uint8)
        _put(r0, o["b"], np.array([0]), "u1")
        _put(r0, o["i1"], np.array([0x7eeeeeee]), "<u4")
        _put(r0, o["i2"], np.array([0xffffffff]), "<u4")
        _put(r0, o["i3"], np.array([0x7ddddddddddddddd], dtype=np.uint64), "<u8")
        _put(r0, o["i4"], np.array([0xfccccccccccccccc], dtype=np.uint64), "<u8")
        _put(r0, o["f1"], np.array([3.141592654], dtype="<f4").view("<u4"), "<u4")
        _put(r0, o["f2"], np.array([2.71828182846], dtype="<f8").view("<u8"), "<u8")
        _put(r0, o["e1"], np.array([1]), "<u4")
        buf[0] = r0[0]
    return buf.reshape(-1), np.zeros(0, dtype=np.uint8)


def rec128(n: int, seed: int = SEED_REC128, first: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """rec128 has the identity layout: field k of the C++ struct is words
    [4k..] / [8k..], so the record is just the draws laid out in order."""
    d = _draws(seed, n, 20, first)
    buf = np.empty((n, 128), dtype=np.uint8)
    buf[:, 0:32] = (d[:, 0:8] & np.uint64(0xFFFFFFFF)).astype("<u4").view(np.uint8).reshape(n, 32)
    buf[:, 32:128] = d[:, 8:20].astype("<u8").view(np.uint8).reshape(n, 96)
    return buf.reshape(-1), np.zeros(0, dtype=np.uint8)


def _payload_bytes(seed: int, n: int, words_per_rec: int, first_word: int, nwords: int,
                   rec0: int = 0) -> np.ndarray:
    """(n, 8*nwords) payload bytes: byte j of a field = byte (j % 8) of
    draw(seed ^ PAYLOAD_XOR, r * words_per_rec + first_word + j // 8)."""
    ps = seed ^ PAYLOAD_XOR
    idx = (np.arange(rec0, rec0 + n, dtype=np.uint64)[:, None] * np.uint64(words_per_rec)
           + np.uint64(first_word) + np.arange(nwords, dtype=np.uint64)[None, :])
    return draw(ps, idx).astype("<u8").view(np.uint8).reshape(n, 8 * nwords)


def _pack_heap(fields: list[tuple[np.ndarray, np.ndarray]]) -> tuple[np.ndarray, list[np.ndarray]]:
    """Pack per-record payload fields into one heap in record order, field
    order.  fields = [(bytes (n, maxlen), lengths (n,)), ...].  Returns the
    heap and, per field, the heap offset of each record's payload."""
    n = fields[0][1].shape[0]
    lens = np.stack([f[1].astype(np.int64) for f in fields], axis=1)  # (n, F)
    flat = lens.reshape(-1)
    starts = np.zeros(flat.shape[0], dtype=np.int64)
    if flat.shape[0] > 1:
        np.cumsum(flat[:-1], out=starts[1:])
    starts = starts.reshape(n, len(fields))
    cols = np.concatenate([f[0] for f in fields], axis=1)
    mask = np.concatenate([np.arange(f[0].shape[1])[None, :] < f[1][:, None] for f in fields],
                          axis=1)
    return cols[mask], [starts[:, k] for k in range(len(fields))]


def _put_ref(buf, off, hoff, lens):
    _put(buf, off, hoff, "<u8")
    _put(buf, off + 8, lens, "<u4")


def recvar(n: int, seed: int = SEED_RECVAR, first: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """Records [first, first + n); heap offsets are relative to this batch's heap."""
    t = S.recvar
    o = t.offsets
    d = _draws(seed, n, 5, first)
    blen = (d[:, 2] % np.uint64(257)).astype(np.int64)
    nlen = (d[:, 3] % np.uint64(65)).astype(np.int64)
    pb = _payload_bytes(seed, n, 40, 0, 40, first)
    blob = pb[:, :256]
    name = (np.uint8(0x61) + pb[:, 256:320] % np.uint8(26)).astype(np.uint8)
    heap, (hb, hn) = _pack_heap([(blob, blen), (name, nlen)])
    buf = np.zeros((n, t.size), dtype=np.uint8)
    _put(buf, o["id"], d[:, 0], "<u8")
    _put(buf, o["kind"], d[:, 1] & np.uint64(0xFFFFFFFF), "<u4")
    _put_ref(buf, o["blob"], hb, blen)
    _put_ref(buf, o["name"], hn, nlen)
    _put(buf, o["score"], d[:, 4], "<u8")
    return buf.reshape(-1), heap


def rpc(n: int, seed: int = SEED_RPC, first: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """rpc_msg records [first, first + n): sel = draw1 % 10; 0-4 CALL,
    5 SUCCESS, 6 PROG_MISMATCH, 7 PROG_UNAVAIL (default void arm),
    8 RPC_MISMATCH, 9 AUTH_ERROR."""
    t = S.rpc_msg
    off = t.offset_of
    d = _draws(seed, n, 16, first)
    sel = (d[:, 1] % np.uint64(10)).astype(np.int64)
    call = sel <= 4
    acc = (sel >= 5) & (sel <= 7)
    den = sel >= 8
    lo32 = lambda x: x & np.uint64(0xFFFFFFFF)  # noqa: E731
    cred_len = np.where(call, (d[:, 6] % np.uint64(401)).astype(np.int64), 0)
    verf_len = np.where(call, (d[:, 8] % np.uint64(401)).astype(np.int64),
                        np.where(acc, (d[:, 6] % np.uint64(41)).astype(np.int64), 0))
    cred_b = _payload_bytes(seed, n, 128, 0, 50, first)
    verf_b = _payload_bytes(seed, n, 128, 64, 50, first)
    heap, (hc, hv) = _pack_heap([(cred_b, cred_len), (verf_b, verf_len)])

    buf = np.zeros((n, t.size), dtype=np.uint8)
    _put(buf, off("xid"), lo32(d[:, 0]), "<u4")
    _put(buf, off("body"), np.where(call, 0, 1).astype(np.uint64), "<u4")

    def put_rows(mask, o, vals, dt):
        if mask.any():
            sub = buf[mask]
            _put(sub, o, vals[mask], dt)
            buf[mask] = sub

    cb = "body.cbody"
    put_rows(call, off(cb + ".rpcvers"), np.full(n, 2, dtype=np.uint64), "<u4")
    put_rows(call, off(cb + ".prog"), lo32(d[:, 2]), "<u4")
    put_rows(call, off(cb + ".vers"), lo32(d[:, 3]), "<u4")
    put_rows(call, off(cb + ".proc"), lo32(d[:, 4]), "<u4")
    put_rows(call, off(cb + ".cred.flavor"), d[:, 5] % np.uint64(2), "<u4")
    put_rows(call, off(cb + ".cred.body"), hc.astype(np.uint64), "<u8")
    put_rows(call, off(cb + ".cred.body") + 8, cred_len.astype(np.uint64), "<u4")
    put_rows(call, off(cb + ".verf.flavor"), d[:, 7] % np.uint64(2), "<u4")
    put_rows(call, off(cb + ".verf.body"), hv.astype(np.uint64), "<u8")
    put_rows(call, off(cb + ".verf.body") + 8, verf_len.astype(np.uint64), "<u4")

    rb = "body.rbody"
    rep = ~call
    put_rows(rep, off(rb), np.where(den, 1, 0).astype(np.uint64), "<u4")
    ar = rb + ".areply"
    put_rows(acc, off(ar + ".verf.flavor"), d[:, 5] % np.uint64(2), "<u4")
    put_rows(acc, off(ar + ".verf.body"), hv.astype(np.uint64), "<u8")
    put_rows(acc, off(ar + ".verf.body") + 8, verf_len.astype(np.uint64), "<u4")
    astat = np.select([sel == 5, sel == 6, sel == 7], [0, 2, 1], 0).astype(np.uint64)
    put_rows(acc, off(ar + ".reply_data"), astat, "<u4")
    pm = sel == 6
    put_rows(pm, off(ar + ".reply_data.mismatch_info.low"), lo32(d[:, 9]), "<u4")
    put_rows(pm, off(ar + ".reply_data.mismatch_info.high"), lo32(d[:, 10]), "<u4")
    rr = rb + ".rreply"
    put_rows(den, off(rr), np.where(sel == 9, 1, 0).astype(np.uint64), "<u4")
    rm = sel == 8
    put_rows(rm, off(rr + ".mismatch_info.low"), lo32(d[:, 9]), "<u4")
    put_rows(rm, off(rr + ".mismatch_info.high"), lo32(d[:, 10]), "<u4")
    ae = sel == 9
    put_rows(ae, off(rr + ".rj_why"), d[:, 11] % np.uint64(15), "<u4")
    return buf.reshape(-1), heap


def vecrec(n: int, seed: int = SEED_VECREC, first: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """Records [first, first + n) of oracle/ref_objects.hh gen_vecrec; each
    element array is staged in the heap 8-byte aligned, in field order."""
    t = S.vecrec
    o = t.offsets
    d = _draws(seed, n, 6, first)
    ps = seed ^ PAYLOAD_XOR
    r = np.arange(first, first + n, dtype=np.uint64)
    nv = (d[:, 1] % np.uint64(17)).astype(np.int64)
    has = (d[:, 2] & np.uint64(1)).astype(np.int64)
    npairs = (d[:, 3] % np.uint64(9)).astype(np.int64)
    flag = ((d[:, 4] >> np.uint64(8)) & np.uint64(1)).astype(np.uint8)
    vals = draw(ps, r[:, None] * np.uint64(32) + np.arange(16, dtype=np.uint64)[None, :])
    vals = (vals & np.uint64(0xFFFFFFFF)).astype("<u4")                  # (n, 16)
    optw = draw(ps, r * np.uint64(32) + np.uint64(16)).astype("<u8")     # low | high << 32
    ph = draw(ps, r[:, None] * np.uint64(32) + np.uint64(17) + np.arange(8, dtype=np.uint64)[None, :])
    pb = ((d[:, 5][:, None] >> np.arange(8, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(np.uint8)
    # element bytes per field, padded to 8 after each array
    vals_b = vals.view(np.uint8).reshape(n, 64)
    opt_b = optw.view(np.uint8).reshape(n, 8)
    pair = np.zeros((n, 8, 16), dtype=np.uint8)
    pair[:, :, 0:8] = ph.astype("<u8").view(np.uint8).reshape(n, 8, 8)
    pair[:, :, 8] = pb
    pair_b = pair.reshape(n, 128)
    lens = np.stack([4 * nv, 8 * has, 16 * npairs], axis=1)              # bytes per array
    padded = (lens + 7) & ~7
    starts = np.zeros(3 * n, dtype=np.int64)
    flat = padded.reshape(-1)
    if flat.size > 1:
        np.cumsum(flat[:-1], out=starts[1:])
    starts = starts.reshape(n, 3)
    cols = np.concatenate([vals_b, opt_b, pair_b], axis=1)              # (n, 200)
    widths = [64, 8, 128]
    mask = np.concatenate([np.arange(w)[None, :] < padded[:, k][:, None] for k, w in enumerate(widths)],
                          axis=1)
    # bytes past an array's length (its 8-byte pad) are zero
    live = np.concatenate([np.arange(w)[None, :] < lens[:, k][:, None] for k, w in enumerate(widths)],
                          axis=1)
    heap = np.where(live, cols, 0).astype(np.uint8)[mask]
    buf = np.zeros((n, t.size), dtype=np.uint8)
    _put(buf, o["id"], d[:, 0] & np.uint64(0xFFFFFFFF), "<u4")
    _put_ref(buf, o["vals"], starts[:, 0], nv)
    _put_ref(buf, o["opt"], starts[:, 1], has)
    _put_ref(buf, o["pairs"], starts[:, 2], npairs)
    _put(buf, o["flag"], flag, "u1")
    return buf.reshape(-1), heap


def containertest(n: int, seed: int = SEED_CONTAINERTEST, first: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """Records [first, first + n) of tests/xdrtest.x containertest (a vector
    of u_4_12 unions, variable-size elements, and bigstr sarr[2]); oracle/
    ref_objects.hh gen_containertest.  d[0..3] = draw(seed, 4r + k):
    nu = d0 % 9 elements, element j takes arm 12 if bit j of d1 is set
    (else 4), its int from payload word 32r + j and its double's bits from
    word 32r + 8 + j; |sarr[0]| = d2 % 33, |sarr[1]| = (d2 >> 32) % 33,
    letters from payload words 32r + 16.. and 32r + 21...  Heap per record:
    the element array (8-byte aligned, 24-byte u_4_12 elements: which, then
    the arm at +8), then the two strings."""
    t, u = S.containertest, S.u_4_12
    o = t.offsets
    ps = seed ^ PAYLOAD_XOR
    d = _draws(seed, n, 4, first)
    r = np.arange(first, first + n, dtype=np.uint64)
    nu = (d[:, 0] % np.uint64(9)).astype(np.int64)
    arm12 = ((d[:, 1][:, None] >> np.arange(8, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
    iv = draw(ps, r[:, None] * np.uint64(32) + np.arange(8, dtype=np.uint64)[None, :]) & np.uint64(0xFFFFFFFF)
    dv = draw(ps, r[:, None] * np.uint64(32) + np.uint64(8) + np.arange(8, dtype=np.uint64)[None, :])
    l0 = (d[:, 2] % np.uint64(33)).astype(np.int64)
    l1 = ((d[:, 2] >> np.uint64(32)) % np.uint64(33)).astype(np.int64)
    s0 = (np.uint8(0x61) + _payload_bytes(seed, n, 32, 16, 5, first) % np.uint8(26)).astype(np.uint8)
    s1 = (np.uint8(0x61) + _payload_bytes(seed, n, 32, 21, 5, first) % np.uint8(26)).astype(np.uint8)
    es = u.size  # 24: which @0, arm @ arms_off (8)
    el = np.zeros((n, 8, es), dtype=np.uint8)
    el[:, :, 0:4] = np.where(arm12, 12, 4).astype("<u4").view(np.uint8).reshape(n, 8, 4)
    ao = u.arms_off
    el[:, :, ao:ao + 4] = iv.astype("<u4").view(np.uint8).reshape(n, 8, 4)
    dd = np.where(arm12, dv, np.uint64(0)).astype("<u8").view(np.uint8).reshape(n, 8, 8)
    el[:, :, ao + S.fix_12.offsets["d"]:ao + S.fix_12.offsets["d"] + 8] = dd
    el = el.reshape(n, 8 * es)
    lens = np.stack([es * nu, l0, l1], axis=1)
    reclen = lens.sum(axis=1)
    starts = np.zeros(n, dtype=np.int64)
    if n > 1:
        np.cumsum((reclen[:-1] + 7) & ~7, out=starts[1:])
    cols = np.concatenate([el, s0, s1], axis=1)                       # (n, 192 + 40 + 40)
    widths = [8 * es, 40, 40]
    live = np.concatenate([np.arange(w)[None, :] < lens[:, k][:, None] for k, w in enumerate(widths)], axis=1)
    # each record's bytes, then zeros up to the next 8-byte boundary
    padw = 8
    pad = np.arange(padw)[None, :] < (((reclen + 7) & ~7) - reclen)[:, None]
    heap = np.concatenate([cols, np.zeros((n, padw), dtype=np.uint8)], axis=1)[
        np.concatenate([live, pad], axis=1)]
    if n:  # no pad after the last record
        heap = heap[:int(starts[-1] + reclen[-1])]
    buf = np.zeros((n, t.size), dtype=np.uint8)
    _put_ref(buf, o["uvec"], starts, nu)
    _put_ref(buf, o["sarr"], starts + es * nu, l0)
    _put_ref(buf, o["sarr"] + 16, starts + es * nu + l0, l1)
    return buf.reshape(-1), heap


def rp_list_nodes(n: int, seed: int = SEED_RP_LIST, first: int = 0) -> np.ndarray:
    """Nodes of lists [first, first + n): 1 + draw(seed, r) % 4, and
    RP_LIST_LONG for r % 65536 == 65535 (oracle/ref_objects.hh rp_list_nodes)."""
    r = np.arange(first, first + n, dtype=np.uint64)
    k = (np.uint64(1) + draw(seed, r) % np.uint64(4)).astype(np.int64)
    k[(r % np.uint64(65536)) == np.uint64(65535)] = RP_LIST_LONG
    return k


def rp_list(n: int, seed: int = SEED_RP_LIST, first: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """Lists [first, first + n) of xdrpp/rpcb_prot.x rp__list (the
    RPCBPROC_DUMP reply, a linked list: one element subroutine per node,
    nested as deep as the list is long); oracle/ref_objects.hh gen_rp_list
    and its stage().  Node g (over the batch from list 0): w0 = draw(ps, 8g),
    w1 = draw(ps, 8g + 1); r_prog = 100000 + w0 % 1000, r_vers = (w0 >> 32)
    % 5; string lengths w1 % 9, (w1 >> 16) % 25, (w1 >> 32) % 13, bytes from
    payload words 8g + 2, 8g + 3.., 8g + 6...  Heap per list, from an 8-byte
    boundary: the strings of every node, then (k > 1) the images of nodes
    1..k-1, 8-byte aligned; node i's rpcb_next = {image of node i + 1, 1}."""
    t = S.rp__list
    stride = t.size  # 72
    om, on = t.offsets["rpcb_map"], t.offsets["rpcb_next"]
    ro = S.rpcb.offsets
    g_first = int(rp_list_nodes(first, seed, 0).sum()) if first else 0
    k = rp_list_nodes(n, seed, first)
    G = int(k.sum())
    ps = seed ^ PAYLOAD_XOR
    g = np.arange(g_first, g_first + G, dtype=np.uint64)
    rec = np.repeat(np.arange(n), k)                         # list of each node
    nstart = np.zeros(n, dtype=np.int64)
    if n > 1:
        np.cumsum(k[:-1], out=nstart[1:])
    pos = np.arange(G) - nstart[rec]                         # node's place in its list
    w0 = draw(ps, np.uint64(8) * g)
    w1 = draw(ps, np.uint64(8) * g + np.uint64(1))
    lens = np.stack([(w1 % np.uint64(9)), (w1 >> np.uint64(16)) % np.uint64(25),
                     (w1 >> np.uint64(32)) % np.uint64(13)], axis=1).astype(np.int64)   # (G, 3)
    words = draw(ps, np.uint64(8) * g[:, None] + np.arange(2, 8, dtype=np.uint64)[None, :])  # (G, 6)
    wb = words.astype("<u8").view(np.uint8).reshape(G, 48)
    cols = np.concatenate([wb[:, 0:8], wb[:, 8:32], wb[:, 32:48]], axis=1)   # netid 8, addr 24, owner 16
    widths = [8, 24, 16]
    # per list: string bytes, then the element images
    sbytes = np.bincount(rec, weights=lens.sum(axis=1), minlength=n).astype(np.int64)
    size = np.where(k > 1, ((sbytes + 7) & ~7) + stride * (k - 1), sbytes)
    H = np.zeros(n, dtype=np.int64)
    if n > 1:
        np.cumsum((size[:-1] + 7) & ~7, out=H[1:])
    total = int(H[-1] + size[-1]) if n else 0
    heap = np.zeros(total, dtype=np.uint8)
    # string offsets: list base + the bytes of the list's earlier strings
    flat = lens.reshape(-1)
    cum = np.zeros(3 * G, dtype=np.int64)
    if flat.size > 1:
        np.cumsum(flat[:-1], out=cum[1:])
    first_piece = cum.reshape(G, 3)[nstart, 0] if n else cum[:0]
    soff = (cum.reshape(G, 3) - first_piece[rec][:, None]) + H[rec][:, None]          # (G, 3)
    live = np.concatenate([np.arange(w)[None, :] < lens[:, j][:, None] for j, w in enumerate(widths)], axis=1)
    dst = np.concatenate([soff[:, j][:, None] + np.arange(w)[None, :] for j, w in enumerate(widths)], axis=1)
    heap[dst[live]] = cols[live]
    # node images
    E = H + ((sbytes + 7) & ~7)                               # list's first element image
    img = np.zeros((G, stride), dtype=np.uint8)
    _put(img, om + ro["r_prog"], (np.uint64(100000) + w0 % np.uint64(1000)), "<u4")
    _put(img, om + ro["r_vers"], ((w0 >> np.uint64(32)) % np.uint64(5)), "<u4")
    for j, f in enumerate(("r_netid", "r_addr", "r_owner")):
        _put_ref(img, om + ro[f], soff[:, j], lens[:, j])
    has_next = pos < (k[rec] - 1)
    _put_ref(img, on, np.where(has_next, E[rec] + stride * pos, 0), has_next.astype(np.int64))
    head = pos == 0
    buf = img[head].reshape(-1).copy()
    rest = ~head
    if rest.any():
        at = E[rec[rest]] + stride * (pos[rest] - 1)
        heap[(at[:, None] + np.arange(stride)[None, :]).reshape(-1)] = img[rest].reshape(-1)
    return buf, heap


GENERATORS = {"numerics": numerics, "rec128": rec128, "recvar": recvar, "rpc": rpc, "vecrec": vecrec,
              "containertest": containertest, "rp_list": rp_list}


def generate(schema: str, n: int, chunk: int = 1 << 16) -> tuple[np.ndarray, np.ndarray]:
    """Generate in chunks (bounded temporaries); heap offsets are rebased."""
    if schema in ("numerics", "rec128") or n <= chunk:
        return GENERATORS[schema](n)
    raise NotImplementedError("chunked generation of var schemas: use generate_var")


# ------------------------------------------------------ RPC call batches
SEED_RPCCALL = 0x5EED0007

# Registered procedures (prog, vers, proc, flags) of the dispatch workload,
# sorted: the servers_ map of rpc_server_base (xdrpp/server.h:218-219) with
# each interface's call_dispatch cases (xdrc/gen_hh.cc:757-774).  Program
# 100005 is an interface with no procedure (flag 1 = XDRG_RPC_PROC_IFACE_ONLY).
RPC_PROCS = np.array(
    [(100000, 2, p, 0) for p in (0, 1, 2, 3, 5, 8)]
    + [(100000, 3, p, 0) for p in range(10)]
    + [(100003, 3, p, 0) for p in range(22)]
    + [(100003, 4, p, 0) for p in range(22)]
    + [(100005, 1, 0, 1)]
    + [(0x20000001, 1, 0, 0)],
    dtype=np.uint32)


def _be(v: np.ndarray) -> np.ndarray:
    """uint32 values -> their XDR (big-endian) words as little-endian uint32."""
    return v.astype(np.uint32).byteswap()


def rpc_calls(n: int, seed: int = SEED_RPCCALL, first: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """A record-marked stream of n RPC messages for the dispatch path
    (SURVEY.md §8 f1).  Returns (stream bytes, offsets[n+1] of the marks).

    Per message i (draws d0..d5 of stream seed, message first+i):
      sel = d2 % 32
        0-23  CALL of a registered procedure (entry d3 % nreal of RPC_PROCS)
        24    rpcvers 3                          -> RPC_MISMATCH reply
        25    d3 odd: unknown prog (0x30000000 + d3 % 1000)  -> PROG_UNAVAIL
              d3 even: prog 100005 (interface with no proc) -> PROC_UNAVAIL
        26    registered prog, vers 100 + d3 % 7  -> PROG_MISMATCH
        27    registered prog/vers, proc 5000 + d3 % 50 -> PROC_UNAVAIL
        28    REPLY (MSG_ACCEPTED, SUCCESS) + result words -> dropped
        29    msg_type 2 + d3 % 5 (bad discriminant) -> malformed
        30    cred body length 401 + d3 % 8 (over opaque<400>) -> malformed
        31    d3 % 3 == 0: truncated after prog (xdr_overflow)
              d3 % 3 == 1: cred length 4k+1..3 with a nonzero pad byte
              d3 % 3 == 2: cred length 0x10000 beyond the message
      xid = lo32(d1); cred flavor d4 % 2, cred length (d4 >> 8) % 101;
      verf flavor 0, verf length (d5 >> 8) % 9; (d5 >> 32) % 25 argument
      words.  Body and argument words are lo32 of draw(seed ^ PAYLOAD_XOR,
      64 * first + word position in the batch), pad bytes zero.
    """
    d = _draws(seed, n, 6, first)
    u = lambda x: x.astype(np.int64)  # noqa: E731
    sel = u(d[:, 2] % np.uint64(32))
    d3 = u(d[:, 3] % np.uint64(1 << 30))
    real = RPC_PROCS[RPC_PROCS[:, 3] == 0]
    ent = real[d3 % len(real)]
    prog, vers, proc = ent[:, 0].astype(np.int64), ent[:, 1].astype(np.int64), ent[:, 2].astype(np.int64)
    rpcvers = np.where(sel == 24, 3, 2)
    s25 = sel == 25
    prog = np.where(s25 & (d3 % 2 == 1), 0x30000000 + d3 % 1000, np.where(s25, 100005, prog))
    vers = np.where(s25 & (d3 % 2 == 0), 1, vers)
    proc = np.where(s25 & (d3 % 2 == 0), d3 % 4, proc)
    vers = np.where(sel == 26, 100 + d3 % 7, vers)
    proc = np.where(sel == 27, 5000 + d3 % 50, proc)
    reply = sel == 28
    mtype = np.where(sel == 29, 2 + d3 % 5, np.where(reply, 1, 0))
    trunc = (sel == 31) & (d3 % 3 == 0)
    badpad = (sel == 31) & (d3 % 3 == 1)
    huge = (sel == 31) & (d3 % 3 == 2)
    cred_len = u((d[:, 4] >> np.uint64(8)) % np.uint64(101))
    cred_len = np.where(sel == 30, 401 + d3 % 8, cred_len)
    cred_len = np.where(badpad, 4 * (cred_len // 8) + 1 + d3 % 3, cred_len)
    cred_wire = np.where(huge, 0, (cred_len + 3) // 4)  # body words present in the stream
    cred_len = np.where(huge, 0x10000, cred_len)
    verf_len = u((d[:, 5] >> np.uint64(8)) % np.uint64(9))
    verf_wire = (verf_len + 3) // 4
    nargs = u((d[:, 5] >> np.uint64(32)) % np.uint64(25))
    # words per message: mark + xid + mtype + [call: 5 + 1 + cred + 2 + verf]
    # or [reply: stat + flavor + len(0) + accept_stat] + args
    call_words = 1 + 1 + 1 + 5 + 1 + cred_wire + 2 + verf_wire + nargs
    reply_words = 1 + 1 + 1 + 4 + nargs
    words = np.where(reply, reply_words, np.where(trunc, 5, call_words))
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(words, out=off[1:])
    total = int(off[-1])
    # every word starts as payload (lo32 of the payload stream, by global word)
    gw = np.arange(total, dtype=np.uint64)
    base = int(first) * 64  # disjoint payload words per message batch position
    out = (draw(seed ^ PAYLOAD_XOR, gw + np.uint64(base)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    o = off[:-1]

    def put(mask, pos, val):
        idx = np.nonzero(mask)[0]
        out[o[idx] + pos[idx] if isinstance(pos, np.ndarray) else o[idx] + pos] = _be(
            np.asarray(val)[idx] if np.ndim(val) else np.full(len(idx), val))

    allm = np.ones(n, dtype=bool)
    put(allm, 0, (words - 1) * 4 | 0x80000000)
    put(allm, 1, d[:, 1] & np.uint64(0xFFFFFFFF))
    put(allm, 2, mtype)
    call = ~reply
    put(call, 3, rpcvers)
    put(call, 4, prog)
    put(call & ~trunc, 5, vers)
    put(call & ~trunc, 6, proc)
    put(call & ~trunc, 7, d[:, 4] % np.uint64(2))
    put(call & ~trunc, 8, cred_len)
    # zero the pad bytes of the last cred / verf word (badpad keeps a nonzero one)
    cl = np.where(call & ~trunc & ~huge & (cred_len % 4 != 0), cred_len, 0)
    m = np.nonzero(cl)[0]
    last = o[m] + 9 + (cl[m] - 1) // 4
    keep = (np.uint64(1) << (np.uint64(8) * (cl[m] % 4).astype(np.uint64))) - np.uint64(1)
    lw = out[last].astype(np.uint64) & keep
    lw = np.where(badpad[m], lw | np.uint64(0xFF000000), lw)
    out[last] = lw.astype(np.uint32)
    vpos = 9 + cred_wire
    put(call & ~trunc, vpos, np.zeros(n, dtype=np.int64))
    put(call & ~trunc, vpos + 1, verf_len)
    vl = np.where(call & ~trunc & (verf_len % 4 != 0), verf_len, 0)
    m = np.nonzero(vl)[0]
    last = o[m] + vpos[m] + 2 + (vl[m] - 1) // 4
    keep = (np.uint64(1) << (np.uint64(8) * (vl[m] % 4).astype(np.uint64))) - np.uint64(1)
    out[last] = (out[last].astype(np.uint64) & keep).astype(np.uint32)
    put(reply, 3, 0)  # MSG_ACCEPTED
    put(reply, 4, 0)  # verf AUTH_NONE
    put(reply, 5, 0)  # verf body<> length 0
    put(reply, 6, 0)  # SUCCESS
    return out.view(np.uint8), (off * 4).astype(np.uint64)
