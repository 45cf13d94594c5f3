"""The product planner (ext_mpi_collectives_amd/csrc/plan.c, via ext_mpi_amd_plan_describe)
against the oracle: replaying the described fold trees on the CPU must reproduce the
oracle's emulation of the reference schedule bit for bit. No GPU needed."""
import numpy as np
import pytest

import ext_mpi_collectives_amd as emac
from helpers import ORACLE_CODE, replay_plan, xorshift_inputs

CONFIGS = [
    (2, "6;1 -2 2"), (2, "6;1 -2"), (2, "6;3 -2 2"), (2, "6;-5 -2 2"),
    (3, "6;1 -3 3"),
    (4, "6;1 -4 4"), (4, "6;1 -2 -2 2 2"), (4, "6;2 -2 -2 4"), (4, "6;-7 -4 4"), (4, "6;1 -2 -2"),
    (6, "6;1 -6 6"), (6, "6;1 -2 -3 3 2"), (6, "6;1 -3 -2 2 3"),
    (8, "6;1 -8 8"), (8, "6;1 -2 -2 -2 2 2 2"), (8, "6;1 -4 -2 2 4"), (8, "6;1 -2 -4 4 2"),
    (8, "6;-64 -8 8"), (8, "6;3 -8 8"), (8, "9;1 -8 8"),
    (12, "6;1 -2 -2 -3 3 2 2"), (16, "6;1 -16 16"), (16, "6;1 -2 -2 -2 -2 2 2 2 2"), (16, "6;1 -4 -4 4 4"),
]
# "1 <members> <level>" sub-splits (reduce_copies_one_socket's multi-level form, reduce_copyin.c:970-1084)
SUBSPLITS = [
    (4, "6;1 -2 2 1 2 1 -2 2"), (6, "6;1 -3 3 1 3 1 -2 2"), (6, "6;1 -2 2 1 2 -4 -3 3"),
    (8, "6;1 -4 4 1 4 1 -2 2"), (8, "6;1 -2 2 1 2 1 -4 4"), (8, "6;1 -2 2 1 2 3 -2 -2 2 2"),
    (8, "6;-3 -2 -2 2 2 1 4 1 -2 2"), (8, "6;1 -2 1 2 -5 -4"), (8, "6;1 -2 2 1 2 1 -2 2 1 2 1 -2 2"),
    (12, "6;1 -3 3 1 3 1 -2 -2 2 2"), (16, "6;1 -4 4 1 4 1 -2 -2 2 2"), (16, "6;-9 -2 -2 2 2 1 4 2 -4 4"),
]
CONFIGS += SUBSPLITS
CODES = [emac.FLOAT, emac.DOUBLE, emac.INT, emac.LONG]


@pytest.mark.parametrize("R,copyin", CONFIGS)
@pytest.mark.parametrize("code", CODES)
def test_plan_replay_equals_oracle(oracle, R, copyin, code):
    for count in (0, 1, 7, 1000, 4099):
        sends = xorshift_inputs(R, count, code)
        want = oracle.allreduce(sends, copyin)
        got = replay_plan(sends, code, copyin)
        for w in want:
            assert np.array_equal(w.view(np.uint8), got.view(np.uint8)), (R, copyin, code, count)


def test_default_copyin_is_linear():
    d = emac.plan_describe(8, 800, emac.FLOAT, None, 3)
    assert d["leaves"] == [3, 0, 1, 2, 4, 5, 6, 7]
    assert d["pieces"] == [(300, 100)] and d["nlev"] == 1


def test_chain_leaf_order():
    # "6;1 -2 -2 -2 2 2 2", owner position 0 (node rank 0): ((s0+s1)+(s2+s3))+((s4+s5)+(s6+s7))
    # in node ranks, per the captured schedule of golden/schedules_survey.json
    d = emac.plan_describe(8, 16384, emac.FLOAT, "6;1 -2 -2 -2 2 2 2", 0)
    assert d["leaves"] == [0, 1, 2, 3, 4, 5, 6, 7]
    assert d["nlev"] == 3
    d5 = emac.plan_describe(8, 16384, emac.FLOAT, "6;1 -2 -2 -2 2 2 2", 5)
    assert d5["owner"] == 5 and d5["pieces"] == [(10240, 2048)]


# copy-in methods 5 (cyclic) / 7 (tree) and their staged aliases 8 / 10, with 1..4 sockets per node
METHODS = [
    (2, "5;1 -2 2", 1), (3, "5;1 -3 3", 1), (4, "5;1 -4 4", 1), (4, "5;1 -2 -2 2 2", 2), (6, "5;1 -2 -3 3 2", 1),
    (6, "5;1 -3 -2 6", 3), (8, "5;1 -4 -2 2 4", 1), (8, "5;3 -2 -4 8", 2), (8, "5;-64 -8 8", 1),
    (8, "8;1 -2 -2 -2 2 2 2", 1), (16, "5;1 -4 -4 4 4", 4), (12, "5;1 -2 -2 -3 3 2 2", 1),
    (2, "7;1 -2 2", 1), (2, "7;1 -2 2", 2), (4, "7;1 -4 4", 1), (4, "7;1 -4 4", 2), (4, "7;1 -2 -2 2 2", 2),
    (6, "7;1 -3 -2 2 3", 2), (6, "7;1 -2 -3 3 2", 3), (8, "7;1 -4 -2 2 4", 2), (8, "7;1 -2 -4 4 2", 4),
    (8, "7;2 -2 -2 -2 2 2 2", 2), (8, "7;-40 -8 8", 1), (8, "10;1 -2 -4 4 2", 2), (12, "7;1 -3 -4 4 3", 4),
    (16, "7;1 -4 -4 4 4", 2), (16, "7;1 -2 -2 -4 4 2 2", 4), (16, "10;1 -16 16", 8),
]


@pytest.mark.parametrize("R,copyin,sockets", METHODS)
@pytest.mark.parametrize("code", CODES)
def test_methods_replay_equals_oracle(oracle, R, copyin, sockets, code):
    for count in (0, 1, 7, 1000, 4099):
        sends = xorshift_inputs(R, count, code)
        want = oracle.allreduce(sends, copyin, num_sockets=sockets)
        got = replay_plan(sends, code, copyin, sockets)
        for w in want:
            assert np.array_equal(w.view(np.uint8), got.view(np.uint8)), (R, copyin, sockets, code, count)


def test_sockets_move_only_the_tree_roots():
    # sockets reach the arithmetic only through the tree's last-step root (reduce_copyin.c:
    # 860-864): recursive and cyclic orders are unchanged, the tree's "-4 -2" order is not
    for copyin in ("6;1 -2 -4 4 2", "5;1 -2 -4 4 2"):
        a = [emac.plan_describe(8, 800, emac.FLOAT, copyin, p)["leaves"] for p in range(8)]
        with emac.num_sockets(4):
            b = [emac.plan_describe(8, 800, emac.FLOAT, copyin, p)["leaves"] for p in range(8)]
        assert a == b
    a = [emac.plan_describe(8, 800, emac.FLOAT, "7;1 -4 -2 2 4", p)["leaves"] for p in range(8)]
    with emac.num_sockets(2):
        b = [emac.plan_describe(8, 800, emac.FLOAT, "7;1 -4 -2 2 4", p)["leaves"] for p in range(8)]
    assert a != b


@pytest.mark.parametrize("bad,sockets", [("7;1 -4", 1), ("7;1 -2 -2", 1), ("5;1 -2 2 1 2 1 -2 2", 1),
                                         ("7;1 -2 2 1 2 1 -2 2", 1), ("7;1 -4 4", 3), ("11;1 -4 4", 1),
                                         ("4;1 -4 4", 1)])
def test_method_limits_rejected(bad, sockets):
    # the tree needs allgather radices (reduce_copyin.c:962-964); cyclic/tree are whole-node
    # generators (no sub-splits); sockets must divide the node; methods outside 5..10
    with emac.num_sockets(sockets):
        with pytest.raises(emac.ExtMpiError):
            emac.plan_describe(4, 100, emac.FLOAT, bad, 0)


def test_set_num_sockets_validates():
    with pytest.raises(emac.ExtMpiError):
        emac.set_num_sockets(0)
    prev = emac.set_num_sockets(2)
    assert emac.set_num_sockets(prev) == 2


@pytest.mark.parametrize("bad", ["6;1 -3 3", "6;1 -2 -2 2", "5;1 -4 -2 2", "6;1 4 -4", "6;1 -4 1 4", "garbage", "6;",
                                 "6;1 -2 2 1 2 1 -4 4", "6;1 -2 2 1 3 1 -2 2", "6;1 -4 4 1 4 1 -1 1"])
def test_invalid_copyin_rejected(bad):
    # (R=4) chain/level size mismatches, a sub-split whose members do not divide the level
    with pytest.raises(emac.ExtMpiError):
        emac.plan_describe(4, 100, emac.FLOAT, bad, 0)


def test_subsplit_equal_pieces_above_a_subsplit_unsupported():
    """reduce_copyin.c:1035-1067 reuse the piece loop's variable inside a sub-split, so the
    reference's generator never terminates for k>1 equal pieces above one: rejected here."""
    with pytest.raises(emac.ExtMpiError):
        emac.plan_describe(8, 100, emac.FLOAT, "6;2 -4 4 1 4 1 -2 2", 0)


def test_subsplit_leaf_order():
    """'6;1 -4 4 1 4 1 -2 2' on 8 ranks: the strided groups {p%2, p%2+2, ...} fold first (own partial,
    then partners ascending), then each contiguous pair folds the two group partials."""
    d = emac.plan_describe(8, 8000, emac.FLOAT, "6;1 -4 4 1 4 1 -2 2", 3)
    # position 3: outer member 1 of group {1,3,5,7}; inner member 1 of block {2,3}
    assert d["leaves"] == [3, 1, 5, 7, 2, 0, 4, 6]
    assert d["nlev"] == 2 and d["pieces"] == [(3000, 1000)]  # outer quarter [2000, 4000), inner half 1


def _radix_chain_copyin(R):
    fs, n = [], R
    for p in (2, 3, 5, 7, 11, 13):
        while n % p == 0:
            fs.append(p)
            n //= p
    return "6;1 " + " ".join(f"-{f}" for f in fs) + " " + " ".join(str(f) for f in reversed(fs)) if len(fs) > 1 else None


def test_layout_accesses_stay_in_bounds():
    """Host replay of every access the fold kernels make (tiles and edge items) for the NODE
    form's buckets: inside [0, count) of every buffer, each destination element written once.
    Random node sizes 1-16, copy-in variants (pieces, -64 fractions, radix chains), element
    counts, types, SUM/MIN/MAX, fan-out 1 or N, and 16-byte phases of every buffer."""
    import ctypes
    import numpy as np
    import ext_mpi_collectives_amd as emac
    f = emac.lib().ext_mpi_amd_check_node_layout
    f.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                  ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    rng = np.random.default_rng(0x1A70)
    tsize = {emac.DOUBLE: 8, emac.LONG: 8, emac.FLOAT: 4, emac.INT: 4}
    for _ in range(1500):
        R = int(rng.integers(1, 17))
        code = int(rng.choice(list(tsize)))
        variants = [f"6;1 -{R} {R}", f"6;-64 -{R} {R}", f"6;{int(rng.integers(2, 6))} -{R} {R}"]
        if _radix_chain_copyin(R):
            variants.append(_radix_chain_copyin(R))
        copyin = variants[int(rng.integers(len(variants)))]
        count = int(min(1 << 17, np.exp(rng.uniform(0, np.log(1 << 17)))))
        phase = (ctypes.c_int * (2 * R))(*[int(x) * tsize[code] for x in rng.integers(0, 16 // tsize[code], 2 * R)])
        op = int(rng.choice([emac.SUM, emac.MIN, emac.MAX]))
        fan = int(rng.integers(0, 2))
        assert f(R, count, code, op, copyin.encode(), phase, fan) == 0, (R, count, code, copyin, list(phase), fan)
