"""CPU: bench.py's own N-rank launcher (`python bench.py --gpus N` without torch.distributed.run).

The driver runs the scaling bench either under torch.distributed.run (WORLD_SIZE set) or as
`python bench.py --gpus N`; in the second form the script must start N ranks itself, before any
GPU call in the parent, and fail when any rank fails or the world size differs from --gpus.
"""
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def test_launch_ranks_starts_n_ranks_with_the_rendezvous_env(tmp_path):
    import bench
    out = tmp_path / "out"
    out.mkdir()
    script = _script(tmp_path, f"""
        import os, sys
        import torch.distributed as dist
        dist.init_process_group("gloo")
        r, w = dist.get_rank(), dist.get_world_size()
        assert os.environ["MASTER_ADDR"] == "127.0.0.1"
        open(os.path.join({str(out)!r}, f"rank{{r}}"), "w").write(f"{{w}} {{' '.join(sys.argv[1:])}}")
        dist.destroy_process_group()
    """)
    assert bench.launch_ranks(2, ["--steps", "3"], script=script) == 0
    got = sorted(os.listdir(out))
    assert got == ["rank0", "rank1"]
    assert all((out / g).read_text() == "2 --steps 3" for g in got)


def test_launch_ranks_reports_a_failing_rank(tmp_path):
    import bench
    script = _script(tmp_path, """
        import os, sys
        sys.exit(3 if os.environ["RANK"] == "1" else 0)
    """)
    assert bench.launch_ranks(2, [], script=script) != 0


def test_gpus_must_match_the_launched_world():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "--gpus 3 but the launcher started 2" in r.stderr
