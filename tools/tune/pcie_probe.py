import sys, json, torch
sys.path.insert(0, "/root/repo")
import bench
dev = torch.device("cuda:0")
for ns in (2, 4, 8):
    for ch in (4 << 20, 16 << 20, 64 << 20):
        print(ns, ch, json.dumps(bench.pcie_ceiling(256 << 20, dev, chunk=ch, nstreams=ns)), flush=True)
