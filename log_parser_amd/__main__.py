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
import sys
from typing import List, Optional

from .utils.config import Config, parse_cli_overrides


def _split(argv: List[str]):
    rest = [a for a in argv if not (a.startswith("-D") and "=" in a)]
    return rest, parse_cli_overrides(argv)


def cmd_validate(args, cfg: Config) -> int:
    from .api import LogParser
    d = args.directory or cfg["pattern.directory"]
    rep = LogParser.from_directory(d, config=cfg.replace({"engine.device": "cpu"})).validate(
        allow=tuple(x for x in args.allow.split(",") if x))
    print(json.dumps({"directory": d, **rep}, indent=2))
    return 1 if any(p["kind"] == "invalid" for p in rep["problems"]) else 0


def cmd_analyze(args, cfg: Config) -> int:
    from .api import LogParser
    if args.patterns:
        cfg = cfg.replace({"pattern.directory": args.patterns})
    if args.device:
        cfg = cfg.replace({"engine.device": args.device})
    lp = LogParser.from_directory(cfg["pattern.directory"], config=cfg)
    out = lp.parse_file(args.file, stream=True if args.stream else None, topk=args.topk, raw=True)
    if isinstance(out, (bytes, bytearray)):
        sys.stdout.buffer.write(out)
        sys.stdout.write("\n")
        return 0
    pats = lp.library.patterns
    top = [{"lineNumber": int(l) + 1, "score": float(s), "patternId": pats[int(p)].id}
           for s, l, p in zip(out.topk_score, out.topk_line, out.topk_pat)]
    print(json.dumps({"totalLines": out.total_lines, "bytes": out.bytes, "chunks": out.chunks,
                      "seconds": round(out.seconds, 3), "summary": out.summary, "topEvents": top}))
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    from .utils.launch import ensure_hw_queues
    ensure_hw_queues()                  # before the first HIP call (profiles/r3_f)
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
