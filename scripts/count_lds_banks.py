#!/usr/bin/env python3
"""LDS bank conflicts of the count-only classification:
rt_scan_kernel<0, 0> reads one byte per position from the 64 KiB class
table t8 at byte address text[i] << 8 | text[i-1] (ds_read_u8; 2 groups of
32 lanes, bank = (address / 4) mod 32, MI355X_MICROARCH.md §LDS).  For
sampled wave-instructions of the kernel's real lane -> position map
(position pc + 256 s + 4 lane + b), the extra LDS cycles (max distinct
dwords on one bank in a group, minus one, summed over the two groups) for
the current layout and for bijective re-layouts: a byte rotation, an xor
of text[i] into the bank bits, and R-way replicated tables.  CPU only."""
import numpy as np, sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import patternmatching_amd as pm
def conflicts(text, addr_fn, trials=2000):
    rng=np.random.default_rng(0)
    tot=0
    for t in range(trials):
        pc = int(rng.integers(1024, len(text)-2048)) & ~1023
        s = int(rng.integers(0,4)); b=int(rng.integers(0,4))
        pos = pc + 256*s + 4*np.arange(64) + b
        key = text[pos].astype(np.uint32) << 8 | text[pos-1]
        A = addr_fn(text[pos].astype(np.uint32), text[pos-1].astype(np.uint32))
        for g in (A[:32], A[32:]):
            words = g >> 2
            bank = words & 31
            # extra cycles = max over banks of distinct words in that bank, minus 1
            m = 0
            for bk in np.unique(bank):
                m = max(m, len(np.unique(words[bank==bk])))
            tot += m-1
    return tot/trials
cur = lambda ti, tp: ti<<8 | tp
def rot(ti,tp):
    W = ti<<24 | tp<<16 | ti<<8 | tp
    return (W >> 6) & 0xFFFF
def xorh(ti,tp):
    return (ti<<8 | tp) ^ ((ti & 31) << 2)
asc = pm.gen_stream(1<<22, 1, 0)
d = pm.Dictionary([__import__('os').path.join(sys.path[0], 'tests', 'golden', 'data', 'snort.dict')])
lines = d.gen_lines(1<<22, 1)
for name, t in (("ascii", asc), ("lines", lines)):
    print(name, "current %.2f rot %.2f xor %.2f extra cycles per wave-instruction" % (conflicts(t, cur), conflicts(t, rot), conflicts(t, xorh)))
def conflicts_rep(text, R, trials=2000, packed=True):
    rng=np.random.default_rng(0)
    tot=0
    lanes=np.arange(64)
    for t in range(trials):
        pc = int(rng.integers(1024, len(text)-2048)) & ~1023
        s = int(rng.integers(0,4)); b=int(rng.integers(0,4))
        pos = pc + 256*s + 4*lanes + b
        key = text[pos].astype(np.uint32) << 8 | text[pos-1]
        d = key >> 4 if packed else key >> 2
        words = d * R + (lanes % R)
        for g in (words[:32], words[32:]):
            bank = g & 31
            m = 0
            for bk in np.unique(bank):
                m = max(m, len(np.unique(g[bank==bk])))
            tot += m-1
    return tot/trials
for name, t in (("ascii", asc), ("lines", lines)):
    print(name, " ".join("R%d %.2f" % (R, conflicts_rep(t, R)) for R in (1,2,4,8)))
def conflicts_repx(text, R, trials=2000):
    rng=np.random.default_rng(0)
    tot=0
    lanes=np.arange(64)
    for t in range(trials):
        pc = int(rng.integers(1024, len(text)-2048)) & ~1023
        s = int(rng.integers(0,4)); b=int(rng.integers(0,4))
        pos = pc + 256*s + 4*lanes + b
        ti = text[pos].astype(np.uint32); tp = text[pos-1].astype(np.uint32)
        key = ti << 8 | tp
        d = (key >> 4) ^ (ti & 31)   # bijection on the word index within the row's 16 words... (ti&31 < 32 ok? d spans 4096)
        words = d * R + (lanes % R)
        for g in (words[:32], words[32:]):
            bank = g & 31
            m = 0
            for bk in np.unique(bank):
                m = max(m, len(np.unique(g[bank==bk])))
            tot += m-1
    return tot/trials
for name, t in (("ascii", asc), ("lines", lines)):
    print(name, "xor", " ".join("R%d %.2f" % (R, conflicts_repx(t, R)) for R in (1,4,8)))
