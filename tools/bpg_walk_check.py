"""Bounds / parity check of the DEVICE one-lane BPG walk on the host (tools/native/bpg_walk_host.cpp
built with AddressSanitizer): the programs of a test library and the lines of its documents, the
text padded like the engine's device buffers. Usage: python tools/bpg_walk_check.py [--seed 3]"""
import argparse
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--no-asan", action="store_true")
    ap.add_argument("--quick", action="store_true", help="one document and 200 random lines (the CPU test)")
    a = ap.parse_args()
    from test_java_shapes import _docs, _shape_library  # noqa: E402

    from log_parser_amd import golden
    from log_parser_amd.models.compiled import CompiledLibrary
    from log_parser_amd.ops.kernels import padded_len
    from log_parser_amd.utils.config import ScoringParams
    from log_parser_amd.native import N
    from test_java_shapes import ALPHA, UNI_PATS, VERDICT_SHAPES
    import random
    sets, trig = _shape_library(a.seed)
    lib = CompiledLibrary(sets, ScoringParams())
    docs = _docs(trig, a.seed)[:1] if a.quick else _docs(trig, a.seed)
    rng = random.Random(a.seed)
    # Unicode / boundary-context shapes as code-point programs, counted repeats, random lines full of
    # non-ASCII code points and terminators next to the documents' lines
    extra = UNI_PATS + VERDICT_SHAPES + [r"X.{0,100}Y", r"a[^\n]{0,40}FATAL", r"(?i)(err|warn).{0,30}x",
                                         r"x{2,40}", r"(?m)^ab.{0,20}c$", r"\bqq.{0,25}zz\b"]
    rand = ["".join(rng.choice(ALPHA + "XYxqz") for _ in range(rng.randint(0, 60))) for _ in range(200 if a.quick else 600)]
    docs = docs + ["\n".join(rand) + "\n"]
    data = "".join(docs).encode("utf-8", errors="surrogatepass")
    lines = golden.split_lines("".join(docs))
    starts, pos = [], 0
    for ln in lines:                               # byte offsets of Java's split("\r?\n") lines
        b = ln.encode("utf-8", errors="surrogatepass")
        starts.append((pos, len(b)))
        pos += len(b)
        if data[pos:pos + 2] == b"\r\n":
            pos += 2
        elif data[pos:pos + 1] == b"\n":
            pos += 1
    tmp = tempfile.mkdtemp()
    progs = [lib.bpg_program(r) for r in lib.bpg_regs]
    for p in extra:
        d = N.compile_regex(p, 2, 4096)              # DFA refused: the code-point program
        if d.get("bpg"):
            progs.append(np.frombuffer(d["bpg"], np.uint64))
    with open(os.path.join(tmp, "progs.bin"), "wb") as f:
        f.write(np.array([len(progs)], np.uint64).tobytes())
        for p in progs:
            f.write(np.array([p.size], np.uint64).tobytes())
            f.write(np.asarray(p, np.uint64).tobytes())
    buf = np.zeros(padded_len(len(data)), np.uint8)
    buf[:len(data)] = np.frombuffer(data, np.uint8)
    buf.tofile(os.path.join(tmp, "text.bin"))
    li = np.array([len(starts)] + [v for s in starts for v in s], np.int64)
    li.tofile(os.path.join(tmp, "lines.bin"))
    exe = os.path.join(tmp, "bpg_walk_host")
    san = [] if a.no_asan else ["-fsanitize=address", "-fno-omit-frame-pointer"]
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", *san, "-I", os.path.join(ROOT, "csrc/kernels"),
                           os.path.join(ROOT, "tools/native/bpg_walk_host.cpp"), "-o", exe])
    r = subprocess.run([exe, *(os.path.join(tmp, x) for x in ("progs.bin", "text.bin", "lines.bin"))])
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
