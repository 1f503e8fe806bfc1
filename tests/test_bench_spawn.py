"""bench.py's own rank launcher (spawn_ranks): `python bench.py --gpus N`
without a launcher starts N rank processes with the torch.distributed
environment set, prints rank 0's line, and exits non-zero when a rank fails
(CPU only: the ranks here are small stand-in scripts)."""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def _bench():
    sys.path.insert(0, ROOT)
    import bench

    return bench


def test_spawn_env_and_rank0_line(tmp_path, capfd):
    s = _script(tmp_path, """
        import json, os, sys
        env = {k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
        if env["RANK"] == "0":
            print(json.dumps(dict(env, argv=sys.argv[1:])))
        """)
    rc = _bench().spawn_ranks(3, ["--gpus", "3", "--steps", "2"], script=s)
    assert rc == 0
    lines = [l for l in capfd.readouterr().out.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["RANK"] == "0" and d["LOCAL_RANK"] == "0" and d["WORLD_SIZE"] == "3"
    assert d["MASTER_ADDR"] == "127.0.0.1" and int(d["MASTER_PORT"]) > 0
    assert d["argv"] == ["--gpus", "3", "--steps", "2"]


def test_spawn_failing_rank_stops_the_others(tmp_path):
    s = _script(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(60)  # would wait in a collective for the failed rank
        """)
    t = time.time()
    rc = _bench().spawn_ranks(2, [], script=s)
    assert rc == 3
    assert time.time() - t < 30


def test_spawn_killed_rank_is_a_failure(tmp_path):
    s = _script(tmp_path, """
        import os, signal
        if os.environ["RANK"] == "1":
            os.kill(os.getpid(), signal.SIGKILL)
        """)
    assert _bench().spawn_ranks(2, [], script=s) != 0


def test_bench_gpus_2_without_gpu_exits_nonzero():
    """The real entry point: with no GPU here every rank fails, so the
    launcher must report failure (and must not hang)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-cpu"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
