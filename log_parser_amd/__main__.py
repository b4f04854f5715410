"""Command line: ``python -m log_parser_amd <command>`` (also installed as ``log-parser-amd``).

  serve     [-Dkey=value ...]                  REST service (POST /parse, Parse.java:23-62)
  analyze   FILE [--patterns DIR] [--stream]   analyse one log file; prints the AnalysisResult
                                               JSON (or a stream summary + top-k for huge logs)
  validate  [DIR]                              compile a pattern library and report every regex
                                               that is invalid, unsupported on the device path,
                                               or routed to the host fallback (the reference only
                                               finds bad regexes per request, AnalysisService.java:64)

Config keys use the reference names (``-Dpattern.directory=...``, env ``PATTERN_DIRECTORY``).
"""
from __future__ import annotations

import argparse
import json
import logging
import mmap
import os
import sys
from typing import List, Optional

from .utils.config import Config, parse_cli_overrides


def _split(argv: List[str]):
    rest = [a for a in argv if not (a.startswith("-D") and "=" in a)]
    return rest, parse_cli_overrides(argv)


def cmd_validate(args, cfg: Config) -> int:
    from .models.compiled import KIND_DFA, KIND_FALLBACK, KIND_INVALID, KIND_NFA, CompiledLibrary
    from .models.library import load_pattern_directory
    d = args.directory or cfg["pattern.directory"]
    sets = load_pattern_directory(d)
    lib = CompiledLibrary(sets, cfg.scoring, max_dfa_states=int(cfg["engine.dfa-max-states"]),
                                  nfa_engine=str(cfg["engine.nfa-engine"]))
    names = {KIND_DFA: "dfa", KIND_NFA: "nfa", KIND_FALLBACK: "host-fallback", KIND_INVALID: "invalid"}
    problems = []
    for r in lib.regexes:
        if r.kind in (KIND_INVALID, KIND_FALLBACK) or (r.kind == KIND_NFA and "nfa" not in args.allow):
            problems.append({"regex": r.pattern, "kind": names.get(r.kind, str(r.kind)), "error": r.error,
                             "roles": sorted(r.roles)})
    out = {"directory": d, "library": lib.summary(), "problems": problems}
    print(json.dumps(out, indent=2))
    return 1 if any(p["kind"] == "invalid" for p in problems) else 0


def cmd_analyze(args, cfg: Config) -> int:
    from .api import LogParser
    if args.patterns:
        cfg = cfg.replace({"pattern.directory": args.patterns})
    if args.device:
        cfg = cfg.replace({"engine.device": args.device})
    lp = LogParser.from_directory(cfg["pattern.directory"], config=cfg)
    size = os.path.getsize(args.file)
    from .parallel.stream import auto_chunk_bytes
    stream = args.stream or size > (int(cfg["engine.chunk-bytes"]) or auto_chunk_bytes(lp.engine.device))
    with open(args.file, "rb") as f:
        if not stream:
            data = f.read()
            sys.stdout.buffer.write(lp.parse_json(data.decode("utf-8", errors="surrogateescape")))
            sys.stdout.write("\n")
            return 0
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) if size else b""
        res = lp.parse_stream(mm, topk=args.topk)
        pats = lp.library.patterns
        top = [{"lineNumber": int(l) + 1, "score": float(s), "patternId": pats[int(p)].id}
               for s, l, p in zip(res.topk_score, res.topk_line, res.topk_pat)]
        print(json.dumps({"totalLines": res.total_lines, "bytes": res.bytes, "chunks": res.chunks,
                          "seconds": round(res.seconds, 3), "summary": res.summary, "topEvents": top}))
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if argv and argv[0] == "serve":
        from .serve.__main__ import main as serve_main
        serve_main(argv[1:])
        return 0
    rest, overrides = _split(argv)
    ap = argparse.ArgumentParser(prog="log-parser-amd", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("serve", help="run the REST service")
    a = sub.add_parser("analyze", help="analyse a log file")
    a.add_argument("file")
    a.add_argument("--patterns", help="pattern directory (default: pattern.directory)")
    a.add_argument("--device", help="cuda | cpu | auto")
    a.add_argument("--stream", action="store_true", help="chunked streaming pass (automatic for big files)")
    a.add_argument("--topk", type=int, default=20)
    v = sub.add_parser("validate", help="compile a pattern library and report problem regexes")
    v.add_argument("directory", nargs="?")
    v.add_argument("--allow", default="nfa", help="comma list of non-DFA kinds not reported (default nfa)")
    args = ap.parse_args(rest)
    logging.basicConfig(level=logging.WARNING, format="%(levelname)s [%(name)s] %(message)s")
    cfg = Config.load(overrides=overrides)
    return {"analyze": cmd_analyze, "validate": cmd_validate}[args.cmd](args, cfg)


if __name__ == "__main__":
    sys.exit(main())
