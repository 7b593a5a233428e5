"""The drop-in's host protocol (include/vpt_run.hpp: drain's taker / pusher / film threads around one staged feed,
run()'s helper threads) over a mock of the C ABI's stream / feed calls, built with ThreadSanitizer
(tests/native/dropin_mock.cpp; no GPU): with 1-3 driving threads, 0-7 helpers, batches of 1-7 tokens, film
snapshots every millisecond, stop_at_next_wave() mid-run, tiny run-ahead bounds (hold / backlog) and the cost
tail on and off, and small frames rendered by jid-range launches instead of a feed, every job id the TileProvider
hands out is rendered exactly once, the host film counts every sample once, and TSan reports no race."""
import os
import subprocess
from pathlib import Path

import pytest

MOCK = Path(__file__).resolve().parent / "native" / "build" / "dropin_mock"

CASES = [
    "drivers=1 helpers=0",
    "drivers=1 helpers=3",
    "drivers=2 helpers=5 batch=3",
    "drivers=3 helpers=2 flush_ms=1 batch=1",
    "drivers=1 helpers=4 stop_after=50 batch=2",
    "drivers=2 helpers=7 batch=1 w=200 h=120 waves=4",
    "drivers=1 helpers=0 hold=100 cost_tail=0 cost_chunks=0 batch=7",
    "drivers=1 helpers=0 hold=5 backlog=3 batch=7 flush_ms=1",
    "drivers=2 helpers=3 hold=37 backlog=11 batch=5 stop_after=90 flush_ms=1",
    # small frames (fewer jobs than the mock's 21 lanes): jid-range launches instead of a feed
    "drivers=1 helpers=0 w=16 h=8 waves=3 batch=2",
    "drivers=3 helpers=0 w=24 h=16 waves=2 batch=1",
    "drivers=1 helpers=0 w=24 h=16 waves=4 stop_after=9 batch=1",
]


@pytest.mark.parametrize("args", CASES)
def test_dropin_protocol_renders_every_token_once(args):
    assert MOCK.exists(), "build with __graft_entry__.build() (tests/native/Makefile)"
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    for _ in range(3):
        r = subprocess.run([str(MOCK), *args.split()], capture_output=True, text=True, timeout=120, env=env)
        assert r.returncode == 0 and "dropin_mock: ok" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
        if "w=16" in args or "w=24" in args:  # the whole frame in direct launches
            assert ", 0 jobs in direct launches" not in r.stdout and "max 0 feeds open" in r.stdout, r.stdout
