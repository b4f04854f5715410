"""Dump real context-DFA tables + a covered-line sample for tools/native/feat_probe.hip, then run it."""
import os
import subprocess
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from log_parser_amd.models.compiled import CompiledLibrary  # noqa: E402
from log_parser_amd.utils.config import ScoringParams  # noqa: E402
from log_parser_amd.utils.synth import make_library, make_log  # noqa: E402

d = "/tmp/fp"
os.makedirs(d, exist_ok=True)
sets, trig = make_library(1000, seed=7)
lib = CompiledLibrary(sets, ScoringParams())
data = make_log(10_000, trig, seed=13, hit_rate=0.01).encode()
lines = data.split(b"\n")
ls = np.cumsum([0] + [len(x) + 1 for x in lines[:-1]]).astype(np.int64)
ll = np.array([len(x) for x in lines], np.int32)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 545
sel = np.linspace(0, len(lines) - 1, n).astype(np.int64)
lib.dfa_meta.astype(np.int32).tofile(f"{d}/meta.bin")
lib.dfa_bytemap.astype(np.uint8).tofile(f"{d}/bm.bin")
lib.dfa_trans.view(np.uint16).tofile(f"{d}/trans.bin")
lib.dfa_acc.astype(np.uint8).tofile(f"{d}/acc.bin")
np.frombuffer(data, np.uint8).tofile(f"{d}/text.bin")
ls[sel].tofile(f"{d}/ls.bin")
ll[sel].tofile(f"{d}/ll.bin")
np.array(lib.ctx_dfa_extent, np.int32).tofile(f"{d}/ext.bin")
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.exit(subprocess.call([os.path.join(root, "tools/bin/feat_probe"), d]))
