"""``python -m log_parser_amd.serve [-Dkey=value ...]`` — run the REST service (port 8080)."""
import logging
import sys

import uvicorn

from ..utils.config import Config, parse_cli_overrides
from .app import create_app


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s [%(name)s] %(message)s")
    cfg = Config.load(overrides=parse_cli_overrides(argv))
    uvicorn.run(create_app(cfg), host=cfg["server.host"], port=int(cfg["server.port"]), log_level="info")


if __name__ == "__main__":
    main()
