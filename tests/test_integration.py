"""The extstore CRC flow of storage.c driven through libmcrc32c.so from C
(tests/integration/storage_sim.c): scalar drop-in on the CPU; batched spill
stamping, page walk + verify and an IO read batch on the GPU.  BASELINE
configs[0] (tests/integration/extstore_config1.c): 10 000 SETs of 4 KiB values
spilled to a page file and read back, checked against the reference's CRCs of
the same items (tests/golden/config1.json)."""
import json
import os
import re
import subprocess

import numpy as np

import pytest

from memcached_amd import build

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    lib = build.build_lib()
    exe = str(tmp_path_factory.mktemp("sim") / "storage_sim")
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(HERE, "integration", "storage_sim.c"), "-L", os.path.dirname(lib), "-lmcrc32c",
                    f"-Wl,-rpath,{os.path.dirname(lib)}", "-o", exe], check=True)
    return exe


def test_storage_sim_scalar_dropin(sim):
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1")  # the CPU leg: batch calls must report ENODEV
    r = subprocess.run([sim], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "scalar drop-in ok" in r.stdout


@pytest.mark.gpu
def test_storage_sim_gpu(sim):
    r = subprocess.run([sim, "--gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "badcrc 1" in r.stdout


@pytest.fixture(scope="module")
def config1_exe(tmp_path_factory):
    lib = build.build_lib()
    exe = str(tmp_path_factory.mktemp("cfg1") / "extstore_config1")
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(HERE, "integration", "extstore_config1.c"), "-L", os.path.dirname(lib), "-lmcrc32c",
                    f"-Wl,-rpath,{os.path.dirname(lib)}", "-o", exe], check=True)
    return exe


def _golden_config1():
    return json.load(open(os.path.join(HERE, "golden", "config1.json")))


def test_config1_extstore_spill_and_readback(config1_exe, tmp_path):
    """Config 1 on the CPU: scalar drop-in for spill and read-back, 0 bad CRCs,
    exactly 1 after one byte is torn on disk, and the spill CRCs of all 10 000
    items identical to the reference crc32c.c's (digest + the page file
    re-checked item by item with the oracle)."""
    from memcached_amd import layout

    from . import oracle
    g = _golden_config1()
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1")
    r = subprocess.run([config1_exe, str(tmp_path)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"config1: (\d+) written in (\d+) wbufs, (\d+) read, badcrc (\d+), torn-item badcrc (\d+), "
                  r"digest ([0-9a-f]{8})", r.stdout)
    assert m, r.stdout
    written, wbufs, read, bad, torn, digest = m.groups()
    assert (int(written), int(wbufs), int(read)) == (g["items"], g["wbufs"], g["items"])
    assert (int(bad), int(torn)) == (0, 1)
    assert int(digest, 16) == g["digest"]
    page = np.fromfile(tmp_path / "extstore.page", np.uint8)
    offs = []
    for w in range(g["wbufs"]):
        o = w * g["wbuf"]
        while o + 48 <= (w + 1) * g["wbuf"] and page[o + layout.NKEY_OFF] != 0:
            offs.append(o)
            o += layout.ntotal_of(page, o)
    offs = np.asarray(offs, np.uint64)
    assert offs.size == g["items"]
    soffs, slens = layout.spans_of(page, offs)
    crcs = oracle.batch(page, soffs, slens)
    stored = page[(offs[:, None] + np.arange(28, 32)).astype(np.int64)].copy().view("<u4").reshape(-1)
    np.testing.assert_array_equal(stored, crcs)
    assert [int(c) for c in crcs[:8]] == g["first_crcs"] and [int(c) for c in crcs[-8:]] == g["last_crcs"]


@pytest.mark.gpu
def test_config1_extstore_batched_gpu(config1_exe, tmp_path):
    """Config 1 with the batched calls: stamp == scalar spill, the page read
    back from the file verifies clean, the 10 000-read batch matches."""
    r = subprocess.run([config1_exe, str(tmp_path), "--gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "config1 gpu: stamped == scalar, page verify nbad 0, read batch mismatches 0" in r.stdout
    assert "digest %08x" % _golden_config1()["digest"] in r.stdout
