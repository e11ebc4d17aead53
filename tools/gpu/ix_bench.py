"""Record index of plain streams (xdrg_index_records) at 1M records per
schema: the speculative walk (index_fast=1) and the list ranking alone
(index_fast=0), beside the decode the index feeds."""
import sys, time, torch
sys.path.insert(0, '.')
from xdrpp_amd import marshal as M, schemas as S, workloads as W
dev = torch.device('cuda:0')


def timed(f, K=10):
    for _ in range(3): r = f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K): r = f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K, r


for name in (sys.argv[1].split(',') if len(sys.argv) > 1 else ['recvar', 'rpc', 'vecrec', 'containertest']):
    n = 1 << 20
    nat, heap = getattr(W, name)(n)
    nat, heap = torch.from_numpy(nat).to(dev), torch.from_numpy(heap).to(dev)
    enc = M.Marshaler(M.Plan(S.ALL[name]), dev).encode(nat, n, heap)
    mar_dec = M.Marshaler(M.Plan(S.ALL[name]), dev)
    dt_dec, _ = timed(lambda: mar_dec.decode(enc.xdr, n, enc.offsets))
    for label, opts in (('fast', {"index_fast": 1}), ('list', {"index_fast": 0})):
        mar = M.Marshaler(M.Plan(S.ALL[name], opts), dev)
        dt, offs = timed(lambda: mar.index_records(enc.xdr, n))
        print(name, label, 'bytes', enc.xdr.numel(), 'index_ms %.3f' % (dt * 1e3),
              'GB/s %.1f' % (enc.xdr.numel() / dt / 1e9), 'decode_ms %.3f' % (dt_dec * 1e3),
              'ratio %.2f' % (dt / dt_dec), 'ok', torch.equal(offs, enc.offsets), flush=True)
