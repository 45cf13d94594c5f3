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
