"""The drop-in PMPI layer (libext_mpi_collectives.so) driven by a plain MPI C program.

CPU (here): the library links, requests it does not own fall through to PMPI, and without a
GPU MPI_Allreduce_init fails loudly (ERROR_DEVICE) instead of reducing on the CPU.
GPU box: one rank (RCCL communicator of size 1) with device and host buffers, in place, with
the reference's known-answer self-test enabled (EXT_MPI_DEBUG=1, the reference default)."""
import os
import shutil
import subprocess

import pytest

import ext_mpi_collectives_amd as emac

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPI_HOME = "/opt/conda"
SRC = os.path.join(ROOT, "tests", "mpi", "mpi_allreduce_check.c")


def _build(tmp_path):
    if not os.path.exists(os.path.join(MPI_HOME, "include", "mpi.h")) or not os.path.exists(emac.MPI_LIB_PATH):
        pytest.skip("MPI headers or the MPI layer are not available")
    exe = str(tmp_path / "mpi_allreduce_check")
    libdir = os.path.dirname(emac.MPI_LIB_PATH)
    # link order: the interception library before libmpi so its strong MPI_* symbols win
    subprocess.run(["gcc", "-O2", SRC, "-o", exe, "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(MPI_HOME, "include"), "-L" + libdir, "-lext_mpi_collectives",
                    "-lext_mpi_amd", os.path.join(MPI_HOME, "lib", "libmpi.so"),
                    # resolve ROCm's libstdc++ needs against the system library, not conda's older one
                    "-Wl,-rpath-link,/lib/x86_64-linux-gnu",
                    "-Wl,-rpath," + libdir, "-Wl,-rpath," + os.path.join(MPI_HOME, "lib")], check=True)
    return exe


def _run(exe, n, args, env=None, timeout=240, cwd=None):
    e = dict(os.environ, **(env or {}))
    p = subprocess.run([os.path.join(MPI_HOME, "bin", "mpiexec"), "-n", str(n), exe] + [str(a) for a in args],
                       capture_output=True, text=True, timeout=timeout, env=e, cwd=cwd)
    out = p.stdout + p.stderr
    return [l for l in out.splitlines() if l.startswith("RESULT")], out


def test_mpi_layer_without_gpu(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu test")
    exe = _build(tmp_path)
    res, out = _run(exe, 2, [1000, "f", "host"])
    assert res and res[0].startswith("RESULT no-device"), out


@pytest.mark.gpu
@pytest.mark.parametrize("args", [[100003, "f", "dev"], [4099, "d", "dev", "inplace"], [100000, "i", "host"],
                                  [777, "l", "host", "inplace"], [0, "f", "dev"]])
def test_mpi_layer_single_rank_gpu(tmp_path, args):
    exe = _build(tmp_path)
    res, out = _run(exe, 1, args, env={"EXT_MPI_DEBUG": "1"})
    assert res and res[0].startswith("RESULT ok"), out


@pytest.mark.parametrize("n,ports,want", [
    (2, None, "RESULT no-device"),               # two logical nodes of 1: the one-port schedule
    (2, "2(-1 1)", "RESULT no-device"),          # the reference's grammar (README, ports_groups.c:55-110)
    (2, "2(-1,1)", "RESULT no-device"),
    (2, "-1 1", "RESULT no-device"),             # a bare port list: one group of that many nodes
    (3, "3(-2 2)", "RESULT no-device"),          # two ports, one radix-3 step
    (3, None, "RESULT no-device"),               # 3 nodes, no list: one radix-3 step
    (4, "4(-3 3)", "RESULT no-device"),
    (4, "4(-1 -1 1 1)", "RESULT no-device"),
    (2, "2(-2 2)", "RESULT fail rc=-4"),         # radix 3 over 2 nodes
    (2, "4(-1 -1 1 1)", "RESULT fail rc=-4"),    # a group of 4 nodes over a communicator of 2
    (2, "-1 -1 1 1", "RESULT fail rc=-4"),       # two steps over 2 nodes
    (2, "2(-1 1) 2(-1 1)", "RESULT fail rc=-4"),  # several groups
    (2, "2(1)", "RESULT no-device"),             # reduction inside the allgather steps (README)
    (4, "4(3)", "RESULT no-device"),
    (4, "4(-1 1 1)", "RESULT no-device"),
    (4, "4(-1 -1)", "RESULT fail rc=-4"),        # reduce_scatter_core: not this path
    (4, "4(-1 2 1)", "RESULT fail rc=-4"),       # an allgather step across the reduce-scatter groups
    (3, "3(-1 1)", "RESULT fail rc=-4"),
])
def test_mpi_logical_nodes_without_gpu(tmp_path, n, ports, want):
    """EXT_MPI_NUM_TASKS_PER_SOCKET splits the ranks into logical nodes (ext_mpi.c:195-215): several
    of them take the inter-node schedule over RCCL (no device here: ERROR_DEVICE on every rank);
    EXT_MPI_NUM_PORTS in the reference's "nodes(ports)" grammar names it, anything else (another
    node count, several groups, a list ending in a reduce-scatter port) is refused
    (ERROR_UNSUPPORTED) instead of computed otherwise."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    exe = _build(tmp_path)
    env = {"EXT_MPI_NUM_TASKS_PER_SOCKET": "1"}
    if ports is not None:
        env["EXT_MPI_NUM_PORTS"] = ports
    res, out = _run(exe, n, [1000, "i", "dev"], env=env)
    assert res and res[0].startswith(want), out


@pytest.mark.parametrize("n,ports,want", [
    (3, "3(-2_2)", "RESULT no-device"),       # one radix-3 step over 3 nodes (ext_mpi_allreduce_blocking_3_1.txt)
    (3, "3(2)", "RESULT no-device"),          # reduction inside the allgather step
    (3, "3(-1_1)", "RESULT pmpi"),            # radix 2 over 3 nodes: PMPI_Allreduce
    (2, "2(-1_1)", "RESULT no-device"),       # the one-port schedule over the 2 nodes: the engine
    (2, "-1_1", "RESULT no-device"),
    (2, "2(-2_2)", "RESULT pmpi"),            # radix 3 over 2 nodes: PMPI_Allreduce
    (2, "4(-1_-1_1_1)", "RESULT pmpi"),       # another node count: PMPI_Allreduce
    (2, "1(-1)", "RESULT pmpi"),              # a one-node row on a two-node communicator
])
def test_mpi_blocking_two_nodes_without_gpu(tmp_path, n, ports, want):
    """Blocking MPI_Allreduce on two logical nodes of one rank reads
    ext_mpi_allreduce_blocking_2_1.txt (<nodes>_<cores per node>, ext_mpi_native_blocking.c:225-230):
    a row naming the one-port schedule over these nodes goes to the engine (ERROR_DEVICE without a
    GPU), any other row to PMPI_Allreduce (checked exact)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    exe = _build(tmp_path)
    (tmp_path / f"ext_mpi_allreduce_blocking_{n}_1.txt").write_text(f"8 1 {ports} 6;1_-1_1\n")
    res, out = _run(exe, n, [1000, "i", "host", "blocking"], cwd=str(tmp_path),
                    env={"EXT_MPI_BLOCKING": "1", "EXT_MPI_NUM_TASKS_PER_SOCKET": "1"})
    assert res and res[0].startswith(want), out


def test_mpi_blocking_without_gpu(tmp_path):
    """EXT_MPI_BLOCKING routes MPI_Allreduce(SUM) to the engine, which fails loudly without a GPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu test")
    exe = _build(tmp_path)
    res, out = _run(exe, 2, [1000, "f", "host", "blocking"], env={"EXT_MPI_BLOCKING": "1"})
    assert res and res[0].startswith("RESULT no-device"), out


# ext_mpi_allreduce_blocking_<nodes>_<cores>.txt as the reference's README shows it: host rows,
# then device rows (the size column restarts); '_' stands for ' ' in the copy-in column.
PARAMS_1_1 = """8 1 1(-1) 9;-64_-1_1
1024 1 1(-1) 6;1_-1_1
8 1 1(-1) 6;-64_-1_1
4096 1 1(-1) 9;1_-1_1
"""


@pytest.mark.gpu
@pytest.mark.parametrize("args,copyin", [
    ([100003, "f", "dev", "blocking"], "9;1 -1 1"),             # 400012 B: device row 2
    ([100, "f", "dev", "blocking"], "6;-64 -1 1"),              # 400 B: device row 1
    ([4099, "d", "dev", "inplace", "blocking"], "9;1 -1 1"),
    ([100, "i", "host", "blocking"], "9;-64 -1 1"),             # 400 B: host row 1
    ([777, "l", "host", "inplace", "blocking"], "6;1 -1 1"),    # 6216 B: host row 2
    ([0, "f", "dev", "blocking"], "9;-64 -1 1"),                # no allocation: host rows
])
def test_mpi_blocking_single_rank_gpu(tmp_path, args, copyin):
    """Blocking MPI_Allreduce: parameter-file row choice, handle cache hits and misses, in place,
    host and device buffers, a derived communicator."""
    exe = _build(tmp_path)
    (tmp_path / "ext_mpi_allreduce_blocking_1_1.txt").write_text(PARAMS_1_1)
    res, out = _run(exe, 1, args, env={"EXT_MPI_BLOCKING": "1", "EXT_MPI_VERBOSE": "1"}, cwd=str(tmp_path))
    assert res and res[0].startswith("RESULT ok"), out
    chosen = [l for l in out.splitlines() if l.startswith("# EXT_MPI blocking allreduce")]
    assert chosen and all(l.endswith("copyin " + copyin) for l in chosen), out


@pytest.mark.gpu
@pytest.mark.parametrize("n,args,extra", [
    (2, [100003, "f", "dev"], {}), (4, [4099, "d", "dev", "inplace"], {}), (3, [100000, "i", "host"], {}),
    (4, [777, "l", "host", "inplace"], {}), (2, [0, "f", "dev"], {}),
    (4, [100003, "f", "dev", "blocking"], {"EXT_MPI_BLOCKING": "1"}),
    (2, [4099, "d", "host", "inplace", "blocking"], {"EXT_MPI_BLOCKING": "1"}),
    (4, [65536, "f", "dev"], {"EXT_MPI_COPYIN": "6;1 -2 -2 2 2"}),
    # the cyclic and tree generators, and two sockets per node (the tree's last roots move)
    (4, [100003, "i", "dev"], {"EXT_MPI_COPYIN": "7;1 -2 -2 2 2", "EXT_MPI_NUM_SOCKETS_PER_NODE": "2"}),
    (4, [65537, "l", "host", "inplace"], {"EXT_MPI_COPYIN": "5;1 -4 4"}),
    (4, [4099, "i", "dev"], {"EXT_MPI_COPYIN": "10;1 -4 4", "EXT_MPI_NUM_SOCKETS_PER_NODE": "2"}),
    # MPI_MIN / MPI_MAX (get_reduction_op, ext_mpi_native.h:77-140): persistent and blocking
    (4, [100003, "d", "dev", "min"], {}), (2, [4099, "i", "host", "inplace", "max"], {}),
    (4, [65536, "l", "dev", "blocking", "max"], {"EXT_MPI_BLOCKING": "1"}),
])
def test_mpi_layer_multi_rank_one_gpu(tmp_path, n, args, extra):
    """n MPI ranks sharing the box's one GPU over the default peer-mapped transport: the
    application's MPI_Allreduce_init / MPI_Start / MPI_Wait (with the known-answer self-test) or
    blocking MPI_Allreduce, checked against PMPI_Allreduce on every rank."""
    exe = _build(tmp_path)
    env = {"EXT_MPI_DEBUG": "1", "EXT_MPI_AMD_BARRIER_TIMEOUT": "20"}
    env.update(extra)
    res, out = _run(exe, n, args, env=env, timeout=180)
    assert res and res[0].startswith("RESULT ok"), out


@pytest.mark.parametrize("env,n,want,printed", [
    ({"EXT_MPI_ALTERNATING": "1", "EXT_MPI_VERBOSE": "1"}, 2, "RESULT no-device", "# EXT_MPI alternating"),
    ({"EXT_MPI_ALTERNATING": "0", "EXT_MPI_VERBOSE": "1"}, 2, "RESULT no-device", "# EXT_MPI not alternating"),
    ({"EXT_MPI_FAST": "1", "EXT_MPI_VERBOSE": "1"}, 2, "RESULT no-device", "# EXT_MPI fast 1"),
    # the non-recursive inter-node generator (allreduce.c) is out of scope: one node unaffected,
    # logical nodes refused (the reference prints the setting whatever EXT_MPI_VERBOSE says)
    ({"EXT_MPI_NOT_RECURSIVE": "1"}, 2, "RESULT no-device", "# EXT_MPI not recursive = 1"),
    ({"EXT_MPI_NOT_RECURSIVE": "1", "EXT_MPI_NUM_TASKS_PER_SOCKET": "1"}, 2, "RESULT fail rc=-4",
     "# EXT_MPI not recursive = 1"),
])
def test_mpi_env_keys_without_gpu(tmp_path, env, n, want, printed):
    """read_env's other keys (ext_mpi.c:58-116) are read on rank 0 and broadcast like the
    reference's: EXT_MPI_ALTERNATING and EXT_MPI_FAST are accepted with nothing to switch (every
    Start is stream-ordered; there is no byte-code interpreter), EXT_MPI_NOT_RECURSIVE refuses
    communicators of several nodes."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    exe = _build(tmp_path)
    res, out = _run(exe, n, [1000, "i", "dev"], env=env)
    assert res and res[0].startswith(want), out
    assert printed in out, out
