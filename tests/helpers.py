"""Test-side helpers: input generators and a numpy replay of the product's described plan."""
import numpy as np

import ext_mpi_collectives_amd as emac

NP = {emac.FLOAT: np.float32, emac.DOUBLE: np.float64, emac.INT: np.int32, emac.LONG: np.int64}
ORACLE_CODE = {emac.DOUBLE: 0, emac.LONG: 1, emac.FLOAT: 2, emac.INT: 3}


def xorshift_inputs(R, count, code, seed_base=0x5EED0000):
    """Per-rank inputs (xorshift64*-style seeded streams per rank).

    float/double uniform in [-1, 1); int in [-2^20, 2^20]; long in [-2^40, 2^40]."""
    out = []
    for r in range(R):
        rng = np.random.Generator(np.random.PCG64(seed_base + r))
        if code in (emac.FLOAT, emac.DOUBLE):
            out.append((rng.random(count) * 2.0 - 1.0).astype(NP[code]))
        elif code == emac.INT:
            out.append(rng.integers(-(1 << 20), (1 << 20) + 1, count, dtype=np.int64).astype(np.int32))
        else:
            out.append(rng.integers(-(1 << 40), (1 << 40) + 1, count, dtype=np.int64))
    return out


def replay_plan(sends, code, copyin, sockets=1):
    """Evaluate the product planner's fold trees (plan_describe) with numpy, element-wise in the
    element type (IEEE round-to-nearest per add, integer wrap)."""
    R = len(sends)
    count = sends[0].size
    out = np.empty_like(sends[0])
    for pos in range(R):
        with emac.num_sockets(sockets):
            d = emac.plan_describe(R, count, code, copyin, pos)
        for off, ln in d["pieces"]:
            if ln <= 0:
                continue
            seg = slice(off, off + ln)
            acc = [None] * max(1, d["nlev"])
            cur = None
            with np.errstate(over="ignore"):
                for t in range(R):
                    cur = sends[d["leaves"][t]][seg]
                    for lvl in range(d["nlev"]):
                        if lvl == 0 or d["close"][t] >= lvl:
                            if (d["first"][t] >> lvl) & 1:
                                acc[lvl] = cur.copy()
                            else:
                                acc[lvl] = acc[lvl] + cur
                        cur = acc[lvl]
            out[seg] = cur
    return out


def ipc_flags_problem(h, world, join_parts=None):
    """None if the peer-mapped handle `h` runs the cross-GPU code exactly when the communicator was
    told to (EXT_MPI_AMD_TEST_CROSS_DEVICE=1: tests on one GPU, whose device UUIDs all match), else
    what differs. The flags (emac.handle_ipc_flags): the agreed cross-device verdict, the
    system-scope release before every phase 0 (engine_ipc.c, engine_join.c), and -- for a fused
    node join (`join_parts` > 1 without EXT_MPI_AMD_JOIN=streams) -- system-scope partial stores,
    i.e. the join_fused_kernel<..., true> instantiation (join_fused.hip)."""
    import os
    cross = os.environ.get("EXT_MPI_AMD_TEST_CROSS_DEVICE", "0") not in ("", "0")
    f = emac.handle_ipc_flags(h)
    want = emac.IPC_CROSS_DEVICE if cross else 0
    if world > 1 and (cross or os.environ.get("EXT_MPI_AMD_IPC_RELEASE", "0") not in ("", "0")):
        want |= emac.IPC_RELEASE_EVENT
    if join_parts and join_parts > 1 and os.environ.get("EXT_MPI_AMD_JOIN") != "streams":
        want |= emac.IPC_SYS_STORES if cross else emac.IPC_DEV_STORES
    return None if f == want else f"ipc flags {f:#x}, want {want:#x}"
