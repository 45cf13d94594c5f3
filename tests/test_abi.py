"""The C-ABI library loads without a GPU and exports every symbol the public headers declare."""
import ctypes
import os
import re

import pytest

import ext_mpi_collectives_amd as emac

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = "\n".join(l for l in text.splitlines() if not l.lstrip().startswith("#"))
    return sorted(set(re.findall(r"\b((?:ext_mpi_amd|EXT_MPI|MPI)_\w+)\s*\(", text)))


def test_core_exports_every_declared_symbol():
    L = emac.lib()
    names = _declared("ext_mpi_amd.h")
    assert len(names) >= 12
    for n in names:
        assert hasattr(L, n), n


def test_mpi_layer_exports_every_declared_symbol():
    if not os.path.exists(emac.MPI_LIB_PATH):
        pytest.skip("MPI layer not built (needs MPI headers)")
    L = ctypes.CDLL(emac.MPI_LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for header in ("ext_mpi_interface.h", "ext_mpi.h"):
        for n in _declared(header):
            assert hasattr(L, n), (header, n)


def test_version_and_no_gpu_error():
    assert "gfx950" in emac.version()
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    # no device: the product fails loudly instead of computing on the CPU
    with pytest.raises(emac.ExtMpiError) as e:
        emac.node_allreduce_init([0, 0], [0, 0], 16, emac.FLOAT)
    assert e.value.code == -5


def test_launch_schedule_policy():
    """emac_gpu_pick_unroll (host code, no GPU): the HBM-tuned node schedule (U = 4, staggered, at
    16 MiB x 8 float), the smallest tile for page-locked host buffers (EMAC_FAN_HOST = 4), the
    wide tile of the one-destination local fold at 32 MiB per leaf, and MIN / MAX on their
    runtime-leaf-count kernel (one vector per lane) whatever the buffers."""
    f = emac.lib().emac_gpu_pick_unroll
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    sched = lambda u, issue: u | issue << 4  # noqa: E731
    nvec = 8 * (2 << 20) // 16  # 8 buckets of 2 MiB
    assert f(emac.SUM, 8, 0, 1, nvec) == sched(4, 5)
    assert f(emac.SUM, 8, 0, 1 | 4, nvec) == sched(1, 1)
    assert f(emac.SUM, 8, 0, 1 | 4, 64) == sched(1, 1)
    assert f(emac.SUM, 8, 0, 1 | 4, 1 << 24) == sched(1, 1)
    assert f(emac.SUM, 8, 1, 1 | 4, nvec) == f(emac.SUM, 8, 1, 1, nvec)  # trees: their own schedule
    assert f(emac.SUM, 8, 0, 0, (32 << 20) // 16) == sched(4, 1)  # local fold, 8 x 32 MiB -> 1
    assert f(emac.SUM, 8, 0, 0, (2 << 20) // 16) == sched(2, 1)
    assert f(emac.SUM, 8, 0, 0, (1 << 20) // 16) == sched(1, 1)
    kremote = 256
    for op in (emac.MIN, emac.MAX):
        assert f(op, 8, 0, 1 | 4, nvec) == f(op, 8, 0, 1, nvec) == f(op, 8, 1, 0, nvec) == sched(1, 1)
        assert f(op, 8, 0, 2, nvec) == sched(1, 1 | kremote)
        assert f(op, 1, 0, 2, nvec) == f(emac.SUM, 1, 0, 2, nvec)  # the IPC pull is a copy whatever the op
