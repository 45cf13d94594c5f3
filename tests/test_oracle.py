"""The oracle (oracle/, a C restatement of the reference) pinned before it is trusted:
against the schedules the reference's generators printed (golden/schedules_survey.json),
against the reference's own known-answer test (golden/kat_*.npz), and against an independent
pure-Python statement of the fold order on small float cases."""
import glob
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
KIND = {0: "SMEMCPY", 1: "SREDUCE"}
BUF = {0: "RECVBUF", 1: "SENDBUF"}


def _ops(oracle, R, rank, nbytes, copyin, stage):
    out = []
    for op in oracle.schedule(R, rank, nbytes, oracle.FLOAT, copyin, stage=stage):
        if op[0] == oracle.OP_PHASE:
            continue
        out.append([KIND[op[0]], BUF[op[1]], op[2], op[3], BUF[op[4]], op[5], op[6], op[7]])
    return out


def test_schedules_match_reference_generators(oracle):
    g = json.load(open(os.path.join(HERE, "golden", "schedules_survey.json")))
    for case in g["cases"]:
        got_in = _ops(oracle, g["nranks"], case["rank"], g["message_bytes"], case["copyin"], 1)
        got_out = _ops(oracle, g["nranks"], case["rank"], g["message_bytes"], case["copyin"], 2)
        if case["complete"]:
            assert got_in == case["copyin_ops"], case["copyin"]
            assert got_out == case["copyout_ops"], case["copyin"]
        else:
            assert got_in[:len(case["copyin_ops"])] == case["copyin_ops"], case["copyin"]


def test_rank_order_radix_chains(oracle):
    # reduce_copyin.c:375-394 applied to the reduce-scatter radices
    assert oracle.rank_order(8, [-2, -2, -2]) == [0, 4, 2, 6, 1, 5, 3, 7]
    assert oracle.rank_order(8, [-4, -2]) == [0, 4, 1, 5, 2, 6, 3, 7]
    assert oracle.rank_order(8, [-8]) == list(range(8))


def test_sizes_displs(oracle):
    # reduce_copyin.c:396-427: remainder on the low ranks; fixed fractions, rest on the last
    s, d = oracle.sizes_displs(4, 4 * 10, 4)
    assert s == [12, 12, 8, 8] and d == [0, 12, 24, 32, 40]
    s, d = oracle.sizes_displs(4, 4 * 10, 4, 3)
    assert s == [12, 12, 12, 4] and d == [0, 12, 24, 36, 40]
    s, d = oracle.sizes_displs(4, 4 * 5, 4, 3)
    assert s == [12, 8, 0, 0]


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(HERE, "golden", "kat_*.npz"))))
@pytest.mark.parametrize("copyin_kind", ["linear", "chain"])
def test_known_answer(oracle, path, copyin_kind):
    f = np.load(path)
    R, count, itemsize, add = (int(x) for x in f["meta"])
    if copyin_kind == "linear":
        copyin = f"6;1 -{R} {R}"
    else:
        copyin = "6;1 " + " ".join(["-2"] * (R.bit_length() - 1) + ["2"] * (R.bit_length() - 1))
    code = oracle.INT if itemsize == 4 else oracle.LONG
    ins = [oracle.kat_fill(count, code, r, add) for r in range(R)]
    for r in range(R):
        assert np.array_equal(ins[r], f["inputs"][r])  # the C fill restates debug_persistent.c
    for out in oracle.allreduce(ins, copyin):
        assert np.array_equal(out, f["expected"])
    for out in oracle.allreduce([x.copy() for x in ins], copyin, in_place=True):
        assert np.array_equal(out, f["expected"])


def _linear_fold_reference(sends, R):
    # pure-Python statement of "6;1 -R R": chunk c is owned by rank c, which copies its own
    # slice then adds ranks 0..R-1 (skipping itself) in ascending order, one at a time.
    n = sends[0].size
    base, extra = divmod(n, R)
    out = np.empty_like(sends[0])
    for c in range(R):
        lo = base * c + min(c, extra)
        hi = lo + base + (c < extra)
        for i in range(lo, hi):
            acc = sends[c][i]
            for j in range(R):
                if j != c:
                    acc = sends[0].dtype.type(acc + sends[j][i])
            out[i] = acc
    return out


@pytest.mark.parametrize("R", [2, 3, 4, 8])
@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_float_fold_order_independent_statement(oracle, R, dt):
    rng = np.random.default_rng(R)
    sends = [(rng.random(203) * 2 - 1).astype(dt) * dt(10.0) ** rng.integers(-3, 4, 203) for _ in range(R)]
    want = _linear_fold_reference(sends, R)
    for out in oracle.allreduce(sends, f"6;1 -{R} {R}"):
        assert np.array_equal(out.view(np.uint8), want.view(np.uint8))


def test_fold_order_is_observable(oracle):
    # the parity tests are only meaningful if different schedules give different float bits
    rng = np.random.default_rng(1)
    sends = [(rng.random(4096) * 2 - 1).astype(np.float32) for _ in range(8)]
    a = oracle.allreduce(sends, "6;1 -8 8")[0]
    b = oracle.allreduce(sends, "6;1 -2 -2 -2 2 2 2")[0]
    assert not np.array_equal(a, b)
    assert np.allclose(a, b, atol=1e-5)


def test_cpu_threads_baseline_matches_emulator(oracle):
    rng = np.random.default_rng(7)
    sends = [(rng.random(10007) * 2 - 1).astype(np.float32) for _ in range(4)]
    recvs = [np.zeros_like(s) for s in sends]
    oracle.cpu_allreduce_threads(sends, recvs, "6;1 -4 4", 3)
    want = oracle.allreduce(sends, "6;1 -4 4")
    for r in range(4):
        assert np.array_equal(recvs[r], want[r])


@pytest.mark.parametrize("copyin", ["6;1 -4 4", "6;1 -2 -2 2 2", "6;-64 -4 4", "6;3 -4 4"])
@pytest.mark.parametrize("dt", [np.float32, np.float64, np.int32, np.int64])
def test_min_max_finite_inputs_are_elementwise_extrema(oracle, copyin, dt):
    # ext_mpi_native_exec.c:240-318 on finite values: any fold order yields the extremum
    rng = np.random.default_rng(11)
    sends = [(rng.integers(-1000, 1000, 3001)).astype(dt) for _ in range(4)]
    for op, ref in ((oracle.MIN, np.minimum.reduce), (oracle.MAX, np.maximum.reduce)):
        want = ref(sends)
        for out in oracle.allreduce(sends, copyin, op=op):
            assert np.array_equal(out, want)


def test_min_max_nan_follows_the_accumulator_rule(oracle):
    # p1 (the owner's accumulator, its own leaf first) takes p2 only if p2 < p1 (MIN) / p2 > p1
    # (MAX); every comparison with NaN is false. So the owner's NaN survives, a partner's NaN
    # never enters: the two owner halves of a 2-rank Allreduce differ.
    sends = [np.full(8, np.nan, np.float32), np.full(8, 1.0, np.float32)]
    for op in (oracle.MIN, oracle.MAX):
        for out in oracle.allreduce(sends, "6;1 -2 2", op=op):
            assert np.isnan(out[:4]).all() and (out[4:] == 1.0).all()
    # signed zeros: -0.0 < +0.0 is false, so the accumulator keeps its own zero
    z = [np.array([0.0, -0.0], np.float64), np.array([-0.0, 0.0], np.float64)]
    out = oracle.allreduce(z, "6;1 -2 2", op=oracle.MIN)[0]
    assert np.signbit(out).tolist() == [False, False]
