"""Diagnostic: unsharded vs sharded(world=1) on a small round; dumps the first package."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pivot-scheduling_amd"), ROOT]
import torch
from oracle import oracle
from pivot_place import synthetic
from pivot_place.engine import PlacementEngine, DeviceRound
mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
r = synthetic.make_round(mode, 5000, 300, seed=1)
eng = PlacementEngine(0)
ref = oracle.place(r)
res = eng.place(r)
print("unsharded equal:", np.array_equal(res.placement, ref.placement))
dr = DeviceRound(r, eng.device)
mx = eng.shard_begin(dr, 0, 5000, 1)
print("max bytes", mx)
send = torch.zeros(mx, dtype=torch.uint8, device=eng.device)
nt, nb = eng.shard_score(send)
torch.cuda.synchronize()
print("nt", nt, "nb", nb)
dt = np.dtype([("s", "<f8"), ("tb", "<u4"), ("id", "<i4")])
pk = send[:nb].cpu().numpy().view(dt).reshape(nt, -1)
print("task0 first 5", pk[0][:5], "bound", pk[0][-1], "valid", (pk[0]["id"] != 0x7fffffff).sum())
try:
    eng.shard_commit(send)
    print("commit ok")
except Exception as e:
    print("commit failed", e)
