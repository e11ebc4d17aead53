import sys, time, torch, numpy as np
sys.path.insert(0, '.')
from xdrpp_amd import marshal as M, schemas as S, workloads as W
dev = torch.device('cuda:0')
for name in ['recvar', 'rpc', 'vecrec']:
    n = 1 << 20
    nat, heap = getattr(W, name)(n)
    nat, heap = torch.from_numpy(nat).to(dev), torch.from_numpy(heap).to(dev)
    mar = M.Marshaler(M.Plan(S.ALL[name]), dev)
    r = mar.encode(nat, n, heap)
    for _ in range(3): offs = mar.index_records(r.xdr, n)
    torch.cuda.synchronize()
    t0 = time.perf_counter(); K = 10
    for _ in range(K): offs = mar.index_records(r.xdr, n)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / K
    print(name, 'bytes', r.xdr.numel(), 'index_ms %.3f' % (dt * 1e3), 'GB/s %.1f' % (r.xdr.numel() / dt / 1e9), 'ok', torch.equal(offs, r.offsets))
