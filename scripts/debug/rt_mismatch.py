"""Debug: RT kernel vs the numpy table emulation on the shipped stream;
prints mismatch statistics (test infrastructure, not product)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import patternmatching_amd as pm
from oracle_lib import DATA, dict_paths
from table_emulator import FlatImage, rt_scan
key = sys.argv[1] if len(sys.argv) > 1 else "et"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
d = pm.Dictionary(dict_paths(key))
img = FlatImage(d.patterns(), pm.KIND_RT)
ship = np.fromfile(os.path.join(DATA, "dictionaries_generated.stream"), dtype=np.uint8)
text = np.tile(ship, reps)
exp = rt_scan(img, text)
m = pm.HipMatcher("rt"); m.add_dictionary(d); m.compile()
got = m.read_block_gids(text)
t12 = img.array("t12").astype(np.uint32)
c0 = text.astype(np.uint32); c1 = np.concatenate([[0], c0[:-1]])
ph = t12[(c0 << 8) | c1] & 0x7FFF
bad = np.nonzero(got != exp)[0]
print(f"{key} n={len(text)} mismatches={len(bad)}")
if len(bad):
    print("got==placeholder", int(np.sum(got[bad] == ph[bad])), "exp==placeholder", int(np.sum(exp[bad] == ph[bad])),
          "got==0", int(np.sum(got[bad] == 0)))
    print("chunk offsets (pos % 1024) hist", np.bincount((bad % 1024) // 128, minlength=8).tolist())
    print("pos % 16 hist", np.bincount(bad % 16, minlength=16).tolist())
    for p in bad[:20]:
        print(int(p), "got", int(got[p]), "exp", int(exp[p]), "ph", int(ph[p]), "bytes", bytes(text[max(0, p - 12):p + 1]))
# device-resident variants: 0 = product, 3 = plain tail
import torch
lib = pm.load()
s = torch.cuda.current_stream()
dt = torch.from_numpy(np.concatenate([text, np.zeros(64, np.uint8)])).cuda()
for var in (0, 3, 4, 5):
    out = torch.zeros(len(text), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    assert lib.pm_hip_debug_scan_variant(m.obj, var, dt.data_ptr(), len(text), out.data_ptr(), 4, cnt.data_ptr(), s.cuda_stream) == 0
    torch.cuda.synchronize()
    g = out.cpu().numpy().astype(np.uint32)
    b2 = np.nonzero(g[1024:-1024] != exp[1024:-1024])[0] + 1024
    print("variant", var, "mismatches", len(b2), "count", int(cnt.item()), "expected count", int(np.count_nonzero(exp)),
          "pos%16", np.bincount(b2 % 16, minlength=16).tolist())
