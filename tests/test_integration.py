"""The extstore CRC flow of storage.c driven through libmcrc32c.so from C
(tests/integration/storage_sim.c): scalar drop-in on the CPU; batched spill
stamping, page walk + verify and an IO read batch on the GPU."""
import os
import subprocess

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
