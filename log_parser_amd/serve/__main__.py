"""``python -m log_parser_amd.serve [-Dkey=value ...]`` — run the REST service (port 8080).

``server.http=native`` (default): the C++ epoll front end (serve/native_http.py);
``server.http=uvicorn``: the FastAPI app under uvicorn (same routes and behaviour)."""
import logging
import signal
import sys
import threading

from ..utils.config import Config, parse_cli_overrides
from .app import Service, create_app


def bind_numa(cfg: Config) -> None:
    """Single-GPU service: run every thread (IO, pump, pipeline) on the CPUs of the GPU's NUMA node,
    before any of them starts -- request bodies, the pinned stage buffers (HIP places them on the
    device's node) and the threads touching them then stay on one socket (``server.numa-bind``)."""
    dev = str(cfg["engine.device"])
    if not cfg.get("server.numa-bind", True) or not dev.startswith("cuda") or cfg.get("engine.serve-devices", ""):
        return
    try:
        import torch
        if not torch.cuda.is_available():
            return
        from ..utils.numa import bind_to_gpu_numa
        cpus = bind_to_gpu_numa(int(dev.split(":", 1)[1]) if ":" in dev else 0)
        if cpus:
            logging.getLogger("log_parser_amd.server").info("bound to the %d CPUs of %s's NUMA node", len(cpus), dev)
    except Exception as e:  # noqa: BLE001 - affinity is an optimisation only
        logging.getLogger("log_parser_amd.server").warning("NUMA binding skipped: %s", e)


def io_threads(cfg: Config, processes: int = 1) -> int:
    """``server.io-threads``, or (0) half of this process's share of the CPU budget, 2..8."""
    n = int(cfg.get("server.io-threads", 0) or 0)
    if n > 0:
        return n
    from ..utils.numa import cpu_budget
    return max(2, min(8, cpu_budget() // (2 * max(processes, 1))))


def raise_fd_limit() -> int:
    """Open-file soft limit up to the hard limit: every keep-alive connection is a descriptor, and
    BASELINE config 5 holds 10k of them at once."""
    try:
        import resource
        soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
        if hard == resource.RLIM_INFINITY or hard > soft:
            resource.setrlimit(resource.RLIMIT_NOFILE, (hard if hard != resource.RLIM_INFINITY else 1 << 20, hard))
        return resource.getrlimit(resource.RLIMIT_NOFILE)[0]
    except (ImportError, ValueError, OSError):
        return -1


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s [%(name)s] %(message)s")
    from ..utils.launch import ensure_hw_queues
    ensure_hw_queues()                  # before the first HIP call (profiles/r3_f)
    cfg = Config.load(overrides=parse_cli_overrides(argv))
    raise_fd_limit()
    from .procs import WorkerContext, process_count, run_processes
    proc = WorkerContext.from_env()
    if proc is None and process_count(cfg) > 1:
        # supervisor of one serving process per GPU (serve/procs.py); makes no HIP call itself
        stop = threading.Event()
        for sig in (signal.SIGINT, signal.SIGTERM):
            signal.signal(sig, lambda *_: stop.set())
        sys.exit(run_processes(argv, cfg, process_count(cfg), stop))
    bind_numa(cfg)
    if str(cfg["server.http"]) == "uvicorn":
        if proc is not None:
            raise SystemExit("server.processes > 1 needs the native HTTP front end (SO_REUSEPORT listeners)")
        import uvicorn
        uvicorn.run(create_app(cfg), host=cfg["server.host"], port=int(cfg["server.port"]), log_level="info")
        return
    from .native_http import NativeHttpFrontend
    stop = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: stop.set())
    fe = NativeHttpFrontend(Service(cfg, proc=proc), cfg["server.host"], int(cfg["server.port"]),
                            io_threads(cfg, proc.nproc if proc is not None else 1))
    fe.serve_forever(stop)


if __name__ == "__main__":
    main()
