"""Literal-verify work of the bloom tier on the bench text (CPU, no GPU): gram hits that reach the
hash table, literal checks they cost (bucket sizes), the largest buckets and the text grams that
hit them. python tools/pf_buckets.py  (profiles/r3_l: 11.6M literal checks per 12.5M-line step)"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, collections
from log_parser_amd.utils.synth import realistic_library, make_log
from log_parser_amd.models.compiled import CompiledLibrary
from log_parser_amd.utils.config import ScoringParams
sets, trig = realistic_library(1000, seed=7)
lib = CompiledLibrary(sets, ScoringParams())
pf = lib.pf
print("stride", pf["stride"], "gmask", pf["gmask"], "lits", len(lib.literals), "teddy", pf["teddy_lits"], "H", pf["ht_mask"]+1)
block = make_log(250_000, trig, seed=11, hit_rate=0.004, aux_rate=0.01, stack_rate=0.01).encode()
a = np.frombuffer(block, np.uint8)
low = a.copy(); m = (low >= 65) & (low <= 90); low[m] += 32
n = len(low) - 4
st = pf["stride"]
pos = np.arange(0, n, st)
g4 = (low[pos].astype(np.uint64) | (low[pos+1].astype(np.uint64) << 8) | (low[pos+2].astype(np.uint64) << 16) | (low[pos+3].astype(np.uint64) << 24))
keys = pf["ht_key"]; cnt = pf["ht_cnt"]
valid = keys != np.uint64(0xFFFFFFFFFFFFFFFF)
tab = {int(k): int(c) for k, c in zip(keys[valid], cnt[valid])}
# exact table hits (g=4 only here; check gmask)
tot = 0; hits = 0; hist = collections.Counter(); gramc = collections.Counter()
for g in (2, 3, 4):
    if not (pf["gmask"] >> g) & 1: continue
    mask = (1 << (8*g)) - 1
    kk = (g4 & np.uint64(mask)) | np.uint64(g << 32)
    u, c = np.unique(kk, return_counts=True)
    for key, k in zip(u.tolist(), c.tolist()):
        b = tab.get(key)
        if b:
            hits += k; tot += k * b; hist[b] += k
            gramc[(key & mask).to_bytes(4, 'little')[:g]] += k
print("lines", block.count(b"\n"), "bytes", len(block), "table gram hits", hits, "literal checks", tot)
print("bucket-size histogram (weighted by hits):", sorted(hist.items())[-10:])
print("top grams:", gramc.most_common(12))
inv = collections.defaultdict(list)
for i, ents in enumerate([]): pass
gl = pf["gram_lits"]; val = pf["ht_val"]
big = [(int(c), int(k)) for k, c, v in zip(keys, cnt, val) if c > 50]
big.sort(reverse=True)
from log_parser_amd.models.compiled import LIT_OFF_SHIFT, MAX_GRAM_OFF
print("MAX_GRAM_OFF", MAX_GRAM_OFF)
for c, k in big[:4]:
    h = list(keys).index(np.uint64(k)); s = int(val[h])
    ls = [lib.literals[int(e) & ((1 << LIT_OFF_SHIFT) - 1)] for e in gl[s:s+c]]
    print(c, (k & 0xFFFFFFFF).to_bytes(4,'little'), ls[:6], min(map(len, ls)), max(map(len, ls)))
