"""``python -m log_parser_amd.serve [-Dkey=value ...]`` — run the REST service (port 8080).

``server.http=native`` (default): the C++ epoll front end (serve/native_http.py);
``server.http=uvicorn``: the FastAPI app under uvicorn (same routes and behaviour)."""
import logging
import signal
import sys
import threading

from ..utils.config import Config, parse_cli_overrides
from .app import Service, create_app


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s [%(name)s] %(message)s")
    cfg = Config.load(overrides=parse_cli_overrides(argv))
    if str(cfg["server.http"]) == "uvicorn":
        import uvicorn
        uvicorn.run(create_app(cfg), host=cfg["server.host"], port=int(cfg["server.port"]), log_level="info")
        return
    from .native_http import NativeHttpFrontend
    stop = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: stop.set())
    fe = NativeHttpFrontend(Service(cfg), cfg["server.host"], int(cfg["server.port"]),
                            int(cfg["server.io-threads"]))
    fe.serve_forever(stop)


if __name__ == "__main__":
    main()
