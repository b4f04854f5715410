import os

import torch

from log_parser_amd.utils.config import Config, env_name, parse_cli_overrides


def test_defaults_match_reference_properties():
    c = Config.load(environ={})
    assert c["pattern.directory"] == "/shared/patterns"
    p = c.scoring
    assert (p.decay_constant, p.max_window) == (10.0, 100)
    assert (p.early_bonus_threshold, p.max_early_bonus, p.penalty_threshold) == (0.2, 2.5, 0.5)
    assert p.max_context_factor == 2.5
    assert (p.freq_threshold, p.freq_max_penalty, p.freq_window_hours) == (10.0, 0.8, 1)


def test_env_mapping_and_precedence(tmp_path):
    props = tmp_path / "application.properties"
    props.write_text("# comment\nscoring.proximity.max-window=50\nscoring.frequency.threshold = 3.5\n")
    env = {"SCORING_FREQUENCY_THRESHOLD": "7"}
    c = Config.load(properties_path=str(props), environ=env)
    assert c.scoring.max_window == 50
    assert c.scoring.freq_threshold == 7.0          # env beats properties
    c2 = Config.load(overrides={"scoring.frequency.threshold": "9"}, properties_path=str(props), environ=env)
    assert c2.scoring.freq_threshold == 9.0         # -D beats env
    assert env_name("scoring.proximity.decay-constant") == "SCORING_PROXIMITY_DECAY_CONSTANT"


def test_cli_overrides():
    assert parse_cli_overrides(["-Dpattern.directory=/x", "foo", "-Da=b=c"]) == {"pattern.directory": "/x", "a": "b=c"}


def test_cpu_budget_and_host_threads(monkeypatch):
    """CPU budget = affinity capped by the cgroup quota; native host threads get 1/n of it per
    serving process (LP_SERVE_NPROC), at most 16."""
    from log_parser_amd.native import host_thread_budget
    from log_parser_amd.utils import numa
    b = numa.cpu_budget()
    assert 1 <= b <= (os.cpu_count() or b)
    monkeypatch.setenv("LP_SERVE_NPROC", "2")
    assert host_thread_budget() == max(1, min(16, b // 2))
    monkeypatch.setattr(numa, "cpu_budget", lambda: 40)
    monkeypatch.setenv("LP_SERVE_NPROC", "1")
    assert host_thread_budget() == 16


def test_registered_empty_falls_back_on_cpu():
    from log_parser_amd.utils.hostmem import registered_empty
    t = registered_empty(4096)
    assert t.numel() == 4096 and t.dtype == torch.uint8 and t.device.type == "cpu"


def test_cpu_limits_and_sched_counters():
    """The config-5 bench's host accounting: affinity / quota limits, cgroup throttling counters
    (empty when the cgroup exposes none) and per-thread run / runqueue-wait nanoseconds."""
    import os
    from log_parser_amd.utils import numa
    from log_parser_amd.utils.restbench import sched_ns
    lim = numa.cpu_limits()
    assert lim["affinity"] >= 1 and (lim["quota_cpus"] is None or lim["quota_cpus"] > 0)
    assert numa.cpu_budget() <= lim["affinity"]
    thr = numa.cgroup_throttling()
    assert thr == {} or set(thr) == {"periods", "throttled_periods", "throttled_ms"}
    run, wait = sched_ns([os.getpid()])
    sum(i * i for i in range(200_000))                # some CPU time on this thread
    run2, wait2 = sched_ns([os.getpid()])
    assert run2 >= run >= 0 and wait2 >= wait >= 0
    assert sched_ns([2 ** 22 + 12345]) == (0, 0)       # no such process
