"""bench.py's multi-GPU launch contract (no GPU needed): --gpus N either runs N ranks
or fails loudly, and the spawned command is one torch.distributed.run on 127.0.0.1."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

import bench  # noqa: E402


def _run(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          env=env, timeout=300)


def test_gpus_beyond_visible_devices_fails_loudly():
    r = _run(["--gpus", "2"])
    assert r.returncode != 0
    assert "requested" in r.stderr and r.stdout == ""


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "3"], {"WORLD_SIZE": "2"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_spawn_command_shape():
    cmd = bench.spawn_command(8, ["--gpus", "8", "--steps", "5"], 12345)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=12345" in cmd
    assert cmd[-3:] == ["--gpus", "8", "--steps", "5"][-3:] and os.path.basename(cmd[-5]) == "bench.py"


def test_per_gpu_work():
    assert bench.packets_per_gpu("uniform", 1) == 1 << 20      # configs[1]
    assert bench.packets_per_gpu("uniform", 8) * 8 == 16 << 20  # configs[3]
    assert bench.packets_per_gpu("large", 8) * 8 == 256 << 10   # configs[4]
    assert bench.packets_per_gpu("uniform", 1, 2 << 20) == 2 << 20


def test_traffic_is_dropped_when_kernel_sources_change(tmp_path, monkeypatch):
    import json

    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_traffic.json").write_text(json.dumps({"uniform": {"hbm_bytes_per_launch": 1.0, "source": "x",
                                                                   "source_hash": "stale"}}))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    assert bench.load_pmc_traffic("uniform") == (None, None)


def test_host_cpus_reports_model_and_threads():
    c = bench.host_cpus()
    assert c["threads"] >= 1 and c["nproc"] >= 1 and isinstance(c["model"], str)


def test_ceiling_fields_frac_of_ceiling():
    """roofline.frac_of_ceiling = the kernel's algorithmic GB/s / the read ceiling measured
    right after the timed steps with the variant that was best before them."""
    import bench

    class FakeCeil:
        def __init__(self):
            self.calls = []

        def measure(self, data, nbytes, launches=10, variants=None):
            self.calls.append((launches, variants))
            return {"gbs": 6400.0, "variant": "nt", "variant_index": 2, "bytes": nbytes, "launches": launches,
                    "variants": {"nt": {"us": 1.0, "gbs": 6400.0}}}

    c = FakeCeil()
    pre = {"gbs": 6500.0, "variant": "nt", "variant_index": 2, "variants": {"nt": {"us": 1.0, "gbs": 6500.0}}}
    f = bench.ceiling_fields(c, pre, None, 1 << 20, 6000.0)
    assert c.calls == [(20, [2])]
    assert f["read_ceiling_gbs"] == 6400.0 and f["frac_of_ceiling"] == round(6000.0 / 6400.0, 4)
    assert f["read_ceiling"]["before_gbs"] == 6500.0 and f["read_ceiling"]["variant"] == "nt"
    none = bench.ceiling_fields(None, None, None, 1, 1.0)
    assert none["read_ceiling_gbs"] is None and none["frac_of_ceiling"] is None
