"""utils/batchlog.py: a batch of per-request INFO lines is written exactly as logging would."""
import io
import logging

from log_parser_amd.utils.batchlog import log_lines


def _capture(fn):
    buf = io.StringIO()
    h = logging.StreamHandler(buf)
    h.setFormatter(logging.Formatter("%(levelname)s [%(name)s] %(message)s"))
    lg = logging.getLogger("lp.test.batchlog")
    lg.handlers[:] = [h]
    lg.setLevel(logging.INFO)
    lg.propagate = False
    fn(lg)
    return buf.getvalue()


def test_log_lines_equals_records():
    lines = ["Received analysis request for pod: a", "Analysis complete for pod: a.", "x %s y"]
    want = _capture(lambda lg: [lg.info("%s", s) for s in lines])
    got = _capture(lambda lg: log_lines(lg, logging.INFO, lines))
    assert got == want and got.count("\n") == 3


def test_log_lines_respects_level():
    assert _capture(lambda lg: log_lines(lg, logging.DEBUG, ["quiet"])) == ""
