"""Pattern-library loader (reference ``PatternService.java:28-95``).

Behaviour kept from the reference:
* recursive walk of ``pattern.directory``; every regular file ending ``.yml``/``.yaml`` is one
  ``PatternSet`` (``PatternService.java:57-63,77-81``);
* a file that fails to parse is logged and skipped (``:82-84``);
* a missing directory is logged and yields zero sets, the service still runs (``:50-55``).

Deliberate difference: files are loaded in sorted path order for determinism
(the reference uses filesystem walk order, which is unspecified).
"""
from __future__ import annotations

import logging
import os
from typing import List

import yaml

from .schema import PatternSet

log = logging.getLogger("log_parser_amd.library")


def load_pattern_file(path: str) -> PatternSet:
    with open(path, "r", encoding="utf-8") as f:
        data = yaml.safe_load(f)
    if data is None:
        data = {}
    if not isinstance(data, dict):
        raise ValueError(f"pattern file {path} does not hold a mapping")
    return PatternSet.model_validate(data)


def load_pattern_directory(directory: str) -> List[PatternSet]:
    log.info("Loading patterns from directory: %s", directory)
    if not directory or not os.path.isdir(directory):
        log.error("Pattern directory does not exist or is not a directory: %s", directory)
        return []
    paths = []
    for root, dirs, files in os.walk(directory):
        dirs.sort()
        for fn in files:
            if fn.endswith(".yml") or fn.endswith(".yaml"):
                p = os.path.join(root, fn)
                if os.path.isfile(p):
                    paths.append(p)
    sets: List[PatternSet] = []
    for p in sorted(paths):
        log.debug("Attempting to load pattern file: %s", p)
        try:
            sets.append(load_pattern_file(p))
        except Exception as e:  # noqa: BLE001 - reference logs and skips any parse failure
            log.error("Failed to parse pattern file: %s (%s)", p, e)
    log.info("Successfully loaded %d pattern sets.", len(sets))
    return sets
