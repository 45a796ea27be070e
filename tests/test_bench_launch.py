"""bench.py's bare N > 1 invocation (`python bench.py --gpus N` without
torchrun's WORLD_SIZE): the parent starts the N ranks under
torch.distributed.run as a child process, before any GPU call, and exits with
the child's status; rank 0's JSON line is the only line on stdout.  CPU only:
a stand-in rank script replaces bench's GPU body."""
import importlib.util
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_launch_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


def test_bare_multi_gpu_invocation_relaunches(monkeypatch):
    b = _bench()
    seen = {}

    def fake(n, argv, script=None):
        seen["n"], seen["argv"] = n, list(argv)
        return 7

    monkeypatch.setattr(b, "relaunch", fake)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    try:
        b.main()
    except SystemExit as e:
        assert e.code == 7
    else:
        raise AssertionError("main() returned instead of exiting with the child's status")
    assert seen == {"n": 4, "argv": ["--gpus", "4", "--steps", "3"]}


def test_relaunch_runs_ranks_and_relays_one_line(tmp_path):
    """The real launcher over gloo on CPU: 2 ranks of a stand-in script that
    checks the torchrun environment and prints bench's line on rank 0 only."""
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent("""
        import json, os, sys
        import torch.distributed as dist
        dist.init_process_group("gloo")
        r, w = dist.get_rank(), dist.get_world_size()
        assert os.environ["MASTER_ADDR"] == "127.0.0.1"
        assert w == int(sys.argv[sys.argv.index("--gpus") + 1])
        dist.barrier()
        if r == 0:
            print(json.dumps({"n_gpus": w, "argv": sys.argv[1:]}), flush=True)
        dist.destroy_process_group()
    """))
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import importlib.util as u; "
            f"s = u.spec_from_file_location('b', {os.path.join(ROOT, 'bench.py')!r}); "
            f"b = u.module_from_spec(s); s.loader.exec_module(b); "
            f"sys.exit(b.relaunch(2, ['--gpus', '2', '--steps', '3'], {str(script)!r}))")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d == {"n_gpus": 2, "argv": ["--gpus", "2", "--steps", "3"]}


def test_relaunch_propagates_failure(tmp_path):
    script = tmp_path / "fail.py"
    script.write_text("import sys; sys.exit(3)\n")
    b = _bench()
    assert b.relaunch(2, [], str(script)) != 0
