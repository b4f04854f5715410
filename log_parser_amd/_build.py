"""Build the native extension ``log_parser_amd/_lpnative.so`` with hipcc for gfx950.

One shared object holds the Java-regex compiler (host C++), the gfx950 kernels with their
host twins (HIP), the JSON emitter and the pybind11 bindings. Objects are rebuilt only when a
source or header is newer than the object. Built in-tree so it travels with the repo snapshot
to the GPU box (see README).
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import sysconfig
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
OUT = os.path.join(ROOT, "log_parser_amd", "_lpnative.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = [
    ("regex/jregex.cpp", "cpp"),
    ("kernels/lp_kernels.hip", "hip"),
    ("kernels/nfa_mfma.hip", "hip"),
    ("kernels/bpg.hip", "hip"),
    ("kernels/scan_multi.hip", "hip"),
    ("kernels/freq_state.hip", "hip"),
    ("kernels/summarize.hip", "hip"),
    ("kernels/line_index.hip", "hip"),
    ("kernels/dp_glue.hip", "hip"),
    ("kernels/lp_post.hip", "hip"),
    ("kernels/post_bulk.hip", "hip"),
    ("kernels/request_io.hip", "hip"),
    ("kernels/side_path.hip", "hip"),
    ("io/json_emit.cpp", "cpp"),
    ("io/docs.cpp", "cpp"),
    ("io/json_in.cpp", "cpp"),
    ("io/http_server.cpp", "cpp"),
    ("io/loadgen.cpp", "cpp"),
    ("runtime/request.cpp", "cpp"),
    ("runtime/proc_shared.cpp", "cpp"),
    ("kernels/prefilter_cpu.cpp", "cpp"),
    ("bind.cpp", "cpp"),
]

_lock = threading.Lock()


def _includes():
    import pybind11
    return ["-I" + CSRC, "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]


def _headers():
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)


def _stale(obj, src, headers):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src] + headers)


def build(verbose: bool = False, force: bool = False) -> str:
    with _lock:
        os.makedirs(BUILD, exist_ok=True)
        headers = _headers()
        objs = []
        procs = []
        # -ffp-contract=off: Java double arithmetic never fuses a*b+c; keep GPU == CPU == reference
        base = ["-O3", "-fPIC", "-pthread", "-std=c++17", "-ffp-contract=off", "-Wno-unused-result", "-D__HIP_PLATFORM_AMD__"]
        for rel, kind in SOURCES:
            src = os.path.join(CSRC, rel)
            if not os.path.exists(src):
                continue
            obj = os.path.join(BUILD, rel.replace("/", "_") + ".o")
            objs.append(obj)
            if not force and not _stale(obj, src, headers):
                continue
            cmd = [HIPCC] + base + _includes()
            if kind == "hip":
                cmd += ["-x", "hip", "--offload-arch=" + ARCH, "-munsafe-fp-atomics"]
            cmd += ["-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd), flush=True)
            procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        for cmd, p in procs:
            out, _ = p.communicate()
            if p.returncode != 0:
                raise RuntimeError("native build failed:\n" + " ".join(cmd) + "\n" + out.decode(errors="replace"))
            if verbose and out:
                sys.stdout.write(out.decode(errors="replace"))
        if force or procs or not os.path.exists(OUT) or any(os.path.getmtime(o) > os.path.getmtime(OUT) for o in objs):
            cmd = [HIPCC, "-shared", "-fPIC", "-pthread", "--offload-arch=" + ARCH] + objs + ["-o", OUT + ".tmp"]
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
            if r.returncode != 0:
                raise RuntimeError("native link failed:\n" + r.stdout.decode(errors="replace"))
            os.replace(OUT + ".tmp", OUT)
        return OUT


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
