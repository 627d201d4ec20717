"""bench.py's measurement fields on the CPU: the traffic record it reports,
the host topology and the reference CPU baseline."""
import json
import os

import numpy as np
import pytest

import bench

from . import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_traffic_is_the_k_fixed_record_of_the_batch_shape():
    """profiles/ holds traffic records of other kernels and shapes
    (r02_traffic_spans.json sorts after r02_traffic.json): the headline takes
    the newest k_fixed record of its own batch shape."""
    t = bench.traffic_per_launch()
    assert t is not None and 1.0 < t / (bench.ITEMS_PER_GPU * bench.ITEM_BYTES) < 1.05
    assert os.path.exists(os.path.join(ROOT, "profiles", "r02_traffic_spans.json"))
    assert bench.traffic_per_launch(items=123) is None


def test_traffic_record_selection(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    rec = {"kernel": "k_fixed", "k1_layout": bench.K1_LAYOUT, "items": 1 << 20, "item_bytes": 4096,
           "hbm_bytes_per_launch": 111.0}
    (prof / "r01_traffic.json").write_text(json.dumps(dict(rec, hbm_bytes_per_launch=100.0)))
    (prof / "r02_traffic.json").write_text(json.dumps(rec))
    (prof / "r02_traffic_spans.json").write_text(json.dumps({"config3": {"traffic_over_algorithmic": 1.02}}))
    (prof / "r03_traffic_other.json").write_text(json.dumps(dict(rec, kernel="k_spans", hbm_bytes_per_launch=9.0)))
    (prof / "r04_traffic_broken.json").write_text("{not json")
    # (a newer record of the earlier K1 layout is not this K1's traffic)
    (prof / "r05_traffic_old_k1.json").write_text(json.dumps(dict(rec, k1_layout="rows32", hbm_bytes_per_launch=5.0)))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.traffic_per_launch(1 << 20, 4096) == 111.0
    assert bench.traffic_per_launch(1 << 19, 4096) is None


def test_cpu_topology_counts_physical_cores():
    cpus, sockets, nlogical, model = bench.cpu_topology()
    assert 1 <= len(cpus) <= nlogical and sockets >= 1 and len(set(cpus)) == len(cpus)
    assert isinstance(model, str) and model


def test_cpu_baseline_runs_the_reference_on_every_core(monkeypatch):
    """The baseline leg on a small batch: the reference crc32c.c (oracle/_ref)
    over the GPU batch's bytes on one pthread per physical core, its CRCs
    equal to the batch's."""
    import torch
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libref_crc32c.so")):
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    n = 512
    rng = np.random.default_rng(3)
    host = rng.integers(0, 256, n * bench.ITEM_BYTES, dtype=np.uint8)
    want = oracle.batch(host, np.arange(n, dtype=np.uint64) * bench.ITEM_BYTES, np.full(n, bench.ITEM_BYTES))
    out = torch.from_numpy(want.view(np.int32).copy())
    r = bench.cpu_baseline(torch.from_numpy(host), out)
    cpus, sockets, _, model = bench.cpu_topology()
    assert r["kind"] == "reference" and r["cores"] == len(cpus) and r["sockets"] == sockets
    assert r["gpu_match"] is True and r["value"] > 0 and r["one_core"] > 0 and r["cpu_model"] == model
    assert r["value"] == max(r["numa_local"], r["resident"])


def test_gpus_n_without_launcher_runs_in_one_process(monkeypatch):
    """`python bench.py --gpus N` (the driver's form, no torchrun) takes the
    single-process path over N devices instead of stopping in dist_setup; with
    fewer visible devices than N it exits with a message naming both counts."""
    import torch
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    called = {}
    monkeypatch.setattr(bench, "headline_devices", lambda a: called.setdefault("n", a.gpus))
    bench.main(["--gpus", "4", "--steps", "3"])
    assert called == {"n": 4}
    monkeypatch.undo()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "2"])
    assert "--gpus 2" in str(e.value) and "1 visible" in str(e.value)


def test_gpus_n_under_a_launcher_keeps_the_rank_path(monkeypatch):
    """Under torchrun (WORLD_SIZE = N) the rank path runs; a WORLD_SIZE that
    differs from --gpus is still an error."""
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(bench, "headline_devices", lambda a: pytest.fail("single-process path taken under a launcher"))
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "4"])
    assert "WORLD_SIZE=2" in str(e.value)
