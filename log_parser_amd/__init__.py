"""log_parser_amd: MI355X-native log-pattern analysis engine (podmortem/log-parser capabilities)."""
__version__ = "0.1.0"


def __getattr__(name):
    if name == "LogParser":
        from .api import LogParser
        return LogParser
    raise AttributeError(name)
