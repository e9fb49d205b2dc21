"""bench.stream_window: the timed window opens on a boundary after the warmup calls and the
settle time, and holds exactly `steps` calls (host logic only, no device)."""
import time

import bench


def _step():
    time.sleep(0.002)
    return [1], None


def test_window_after_settle_on_boundary():
    t = time.perf_counter()
    win = bench.stream_window(_step, [1], 4, 8, 4, settle_s=0.05, boundary=4)
    w = win["warm_calls"]
    assert w % 4 == 0 and w >= 4
    assert len(win["latencies"]) == 8
    # the window opened no earlier than the settle time
    assert time.perf_counter() - t >= 0.05
    assert win["calls_total"] >= w + 8


def test_window_without_settle_keeps_warmup_count():
    win = bench.stream_window(_step, [1], 6, 5, 3)
    assert win["warm_calls"] == 6 and len(win["latencies"]) == 5
    win = bench.stream_window(_step, [1], 0, 5, 3)
    assert win["warm_calls"] == 0 and len(win["latencies"]) == 5


def test_geometry_is_the_library_default_whatever_the_steps(monkeypatch):
    monkeypatch.delenv("BGV_MAX_BATCH_SLOTS", raising=False)
    # 131,072 default slots: 16 calls of 8192 sets, for the driver's --steps 20 and the default 64
    assert bench.super_batch_calls(8192) == 16
    assert bench.super_batch_calls(1024) == 128
    monkeypatch.setenv("BGV_MAX_BATCH_SLOTS", "65536")
    assert bench.super_batch_calls(8192) == 8


def test_timed_calls_cover_whole_completion_periods():
    # period = 16 calls x 2 dispatchers: 20 requested steps time one whole period, 64 exactly two
    assert bench.timed_calls(20, 16, 2) == 32
    assert bench.timed_calls(64, 16, 2) == 64
    assert bench.timed_calls(65, 16, 2) == 96
    assert bench.timed_calls(1, 1, 2) == 2
