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
@pytest.mark.parametrize("copyin_kind", ["linear", "chain", "cyclic", "cyclic_chain", "tree", "tree2s", "staged"])
def test_known_answer(oracle, path, copyin_kind):
    # the known answer holds for every copy-in method (5 cyclic, 6 recursive, 7 tree; 8-10 the
    # same on a staging copy) and for two sockets per node
    f = np.load(path)
    R, count, itemsize, add = (int(x) for x in f["meta"])
    k = R.bit_length() - 1
    chain = " ".join(["-2"] * k + ["2"] * k)
    copyin, sockets = {"linear": (f"6;1 -{R} {R}", 1), "chain": ("6;1 " + chain, 1),
                       "cyclic": (f"5;1 -{R} {R}", 1), "cyclic_chain": ("5;1 " + chain, 2),
                       "tree": ("7;1 " + chain, 1), "tree2s": ("7;1 " + chain, 2),
                       "staged": (f"10;2 -{R} {R}", 1)}[copyin_kind]
    code = oracle.INT if itemsize == 4 else oracle.LONG
    ins = [oracle.kat_fill(count, code, r, add) for r in range(R)]
    for r in range(R):
        assert np.array_equal(ins[r], f["inputs"][r])  # the C fill restates debug_persistent.c
    for out in oracle.allreduce(ins, copyin, num_sockets=sockets):
        assert np.array_equal(out, f["expected"])
    for out in oracle.allreduce([x.copy() for x in ins], copyin, in_place=True, num_sockets=sockets):
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


@pytest.mark.parametrize("R,sockets", [(2, 2), (4, 2), (6, 2), (6, 3), (8, 2), (8, 4), (12, 3), (16, 2), (16, 4)])
def test_get_rank_cyclic_decodes_to_the_node_rank(oracle, R, sockets):
    # reduce_copyin.c:482-486 encodes a peer position as a buffer-table index; the table of
    # ext_mpi_xpmem.c:114-130 (socket-base rotation, then a per-socket rotation) must decode it
    # to the peer's node rank for every rank order the generators use
    for ranks in (list(range(R)), oracle.rank_order(R, [-2] * (R.bit_length() - 1)) if R & (R - 1) == 0
                  else list(range(R))[::-1]):
        for me in range(R):
            for other in range(R):
                idx = oracle.get_rank_cyclic(sockets, R, ranks, me, other)
                assert 0 <= idx < R
                assert oracle.decode_peer(sockets, R, ranks[me], idx) == ranks[other]
                # with one socket the encoding is the plain rank difference
                assert oracle.get_rank_cyclic(1, R, ranks, me, other) == (ranks[other] - ranks[me]) % R


def _chunks(oracle, n, R, f0, itemsize):
    """element ranges [lo, hi) of chunk j of every piece (reduce_copyin.c:396-427, :1035-1081)"""
    pieces = []
    if f0 < 0:
        s, d = oracle.sizes_displs(R, n * itemsize, itemsize, -f0)
        return [[(d[j] // itemsize, (d[j] + s[j]) // itemsize) for j in range(R)]]
    base, extra = divmod(n, f0)
    first = 0
    for i in range(f0):
        ln = base + (i < extra)
        s, d = oracle.sizes_displs(R, ln * itemsize, itemsize)
        pieces.append([(first + d[j] // itemsize, first + (d[j] + s[j]) // itemsize) for j in range(R)])
        first += ln
    return pieces


def _fold(vals):
    acc = vals[0].copy()
    for v in vals[1:]:
        acc = (acc + v).astype(acc.dtype)
    return acc


def _cyclic_statement(sends, R, rs):
    """Method 5 (reduce_copyin.c:531-634) as algebra: after step s, position p holds for chunk
    c in [p, p + gb_s) the left fold [own, p - gb_s, p - 2 gb_s, ...] of the step s-1 partials;
    chunk c ends complete at position c. Identity rank order. Returns value(c) callables."""
    gbs = [int(np.prod(rs[s + 1:])) for s in range(len(rs))]

    def v(s, p, c, lo, hi):
        if s < 0:
            return sends[p][lo:hi]
        return _fold([v(s - 1, (p - gbs[s] * q) % R, c, lo, hi) for q in range(rs[s])])
    return lambda c, lo, hi: v(len(rs) - 1, c, c, lo, hi)


def _tree_statement(sends, R, rs, ranks, sockets):
    """Method 7 (reduce_copyin.c:844-968) as algebra over positions: step s folds, into the
    buffer of root = gb_s * sock + r, the step s-1 partials of positions gb_s * q + r (root
    first, then q != sock ascending); sock = p / (R / |f_s|) at gb_s == 1 with several sockets."""
    gbs = [int(np.prod(rs[s + 1:])) for s in range(len(rs))]

    def sock(s, p):
        return p // (R // rs[s]) if sockets > 1 and gbs[s] == 1 else 0

    def v(s, rho, j, lo, hi):
        if s < 0:
            return sends[ranks[rho]][lo:hi]
        gb = gbs[s]
        r = rho % gb
        k = sock(s, (j // gb) * gb + r)
        assert rho == gb * k + r
        return _fold([v(s - 1, rho, j, lo, hi)] + [v(s - 1, gb * q + r, j, lo, hi) for q in range(rs[s]) if q != k])
    last = len(rs) - 1
    return lambda j, lo, hi: v(last, sock(last, j), j, lo, hi)


@pytest.mark.parametrize("copyin,R,sockets", [
    ("5;1 -4 4", 4, 1), ("5;1 -2 -2 2 2", 4, 1), ("5;1 -2 -3 3 2", 6, 1), ("5;1 -2 -2 -2 2 2 2", 8, 2),
    ("5;3 -4 -2 8", 8, 1), ("5;-40 -4 4", 4, 1), ("8;1 -3 -2 6", 6, 1),
    ("7;1 -2 -2 2 2", 4, 1), ("7;1 -2 -2 -2 2 2 2", 8, 1), ("7;1 -2 -2 -2 2 2 2", 8, 2), ("7;1 -4 -2 2 4", 8, 2),
    ("7;1 -2 -4 4 2", 8, 4), ("7;1 -3 -2 2 3", 6, 2), ("7;1 -3 -2 2 3", 6, 3), ("7;2 -2 -2 2 2", 4, 1),
    ("10;1 -2 -3 3 2", 6, 3), ("7;1 -8 8", 8, 1)])
@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_cyclic_and_tree_fold_order_independent_statement(oracle, copyin, R, sockets, dt):
    method, factors = oracle.parse_copyin(copyin)
    base = method - 3 if method >= 8 else method
    rs = [-f for f in factors[1:] if f < 0]
    rng = np.random.default_rng(R * 31 + len(rs))
    n = 397
    sends = [((rng.random(n) * 2 - 1) * 10.0 ** rng.integers(-3, 4, n)).astype(dt) for _ in range(R)]
    if base == 5:
        value = _cyclic_statement(sends, R, rs)
    else:
        ranks = oracle.rank_order(R, [f for f in factors[1:] if f < 0])
        value = _tree_statement(sends, R, rs, ranks, sockets)
    want = np.empty(n, dt)
    for piece in _chunks(oracle, n, R, factors[0], np.dtype(dt).itemsize):
        for j, (lo, hi) in enumerate(piece):
            if hi > lo:
                want[lo:hi] = value(j, lo, hi)
    for out in oracle.allreduce(sends, copyin, num_sockets=sockets):
        assert np.array_equal(out.view(np.uint8), want.view(np.uint8)), copyin
    for out in oracle.allreduce([x.copy() for x in sends], copyin, in_place=True, num_sockets=sockets):
        assert np.array_equal(out.view(np.uint8), want.view(np.uint8)), copyin


def test_methods_give_distinct_fold_orders(oracle):
    # the cyclic and tree parity tests only bite if their bits differ from method 6's (radix-2
    # steps are commutative single adds, so only radices > 2 separate the orders; the socket
    # count moves the tree's last-step roots, visible with a last radix > 2)
    rng = np.random.default_rng(3)
    sends = [(rng.random(4096) * 2 - 1).astype(np.float32) for _ in range(8)]
    outs = {c: oracle.allreduce(sends, c, num_sockets=s)[0] for c, s in
            (("6;1 -4 -2 2 4", 1), ("5;1 -4 -2 2 4", 1), ("7;1 -4 -2 2 4", 1), ("7;1 -2 -4 4 2", 1),
             ("7;1 -2 -4 4 2", 4))}
    keys = list(outs)
    for i in range(len(keys)):
        for j in range(i + 1, len(keys)):
            assert not np.array_equal(outs[keys[i]], outs[keys[j]]), (keys[i], keys[j])


def test_tree_without_allgather_radices_is_rejected(oracle):
    # reduce_copyin.c:962-964: "reduce_copies_tree not implemented"
    sends = [np.ones(16, np.float32)] * 4
    with pytest.raises(ValueError):
        oracle.allreduce(sends, "7;1 -4")


@pytest.mark.parametrize("R,copyin", [(1, "6;1 -1 1"), (2, "6;1 -2 2"), (4, "6;1 -2 -2 2 2"), (4, "7;1 -4 4"),
                                      (8, "5;1 -8 8")])
def test_two_nodes_known_answer(oracle, R, copyin):
    # ext_mpi_native.c:879-1000 + allreduce_recursive.c:222-453 (one port): integer sums over both
    # nodes' ranks exactly, in place and out of place
    W = 2 * R
    for count, code in ((1000, oracle.INT), (777, oracle.LONG)):
        ins = [oracle.kat_fill(count, code, r, 73) for r in range(W)]
        want = np.sum(np.stack(ins).astype(np.int64), axis=0).astype(ins[0].dtype)
        for in_place in (False, True):
            for out in oracle.allreduce_nodes([x.copy() for x in ins], copyin, 2, in_place=in_place):
                assert np.array_equal(out, want)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_two_nodes_fold_is_one_reduction_of_the_node_partials(oracle, dt):
    # every element = (node 0's single-node result) + (node 1's): one two-operand add, commutative
    rng = np.random.default_rng(5)
    R = 4
    sends = [((rng.random(1003) * 2 - 1) * 10.0 ** rng.integers(-3, 4, 1003)).astype(dt) for _ in range(2 * R)]
    p0 = oracle.allreduce(sends[:R], "6;1 -4 4")[0]
    p1 = oracle.allreduce(sends[R:], "6;1 -4 4")[0]
    for out in oracle.allreduce_nodes(sends, "6;1 -4 4", 2):
        assert np.array_equal(out, (p0 + p1).astype(dt)) and np.array_equal(out, (p1 + p0).astype(dt))


def test_many_nodes_pairwise_tree(oracle):
    # 4 nodes, one port per step: allreduce_core pairs task t with t ^ 2 then t ^ 1
    # (allreduce_recursive.c:261-284). The tasks are NOT ext_mpi_rank_order's [0, 2, 1, 3]: the
    # forward permutation pass discards that RANK_PERM (rank_permutation.c:90,106) and runs with
    # the identity when the 4 lines are equal -- ((P0 + P2) + (P1 + P3)) -- else with
    # rank_perm_heuristic over the line sizes: 517 = 130 + 3 x 129 gives [2, 3, 1, 0], so
    # ((P2 + P1) + (P3 + P0)).
    rng = np.random.default_rng(9)
    f32 = np.float32
    for count, pairs in ((516, ((0, 2), (1, 3))), (517, ((2, 1), (3, 0)))):
        sends = [((rng.random(count) * 2 - 1) * 10.0 ** rng.integers(-4, 5, count)).astype(f32) for _ in range(8)]
        p = [oracle.allreduce(sends[2 * n:2 * n + 2], "6;1 -2 2")[0] for n in range(4)]
        (a, b), (c, d) = pairs
        want = ((p[a] + p[b]).astype(f32) + (p[c] + p[d]).astype(f32)).astype(f32)
        other = ((p[0] + p[1]).astype(f32) + (p[2] + p[3]).astype(f32)).astype(f32)
        assert not np.array_equal(want, other)  # the pairing is observable
        for out in oracle.allreduce_nodes(sends, "6;1 -2 2", 4):
            assert np.array_equal(out, want)
    assert _perm_heuristic(4, [130, 129, 129, 129]) == [2, 3, 1, 0]


def _rank_order(size, factors, ranks):
    """ext_mpi_rank_order (reduce_copyin.c:375-394), literally: the permutation lands in `ranks`
    only through the recursive copy-back (:383-393), so a single factor leaves `ranks` as it is."""
    if len(factors) <= 1:
        return list(ranks)
    f0, blk = abs(factors[0]), size // abs(factors[0])
    new = [0] * size
    for i in range(blk):
        for j in range(f0):
            new[i + j * blk] = ranks[i * f0 + j]
    for j in range(f0):
        new[j * blk:(j + 1) * blk] = _rank_order(blk, factors[1:], new[j * blk:(j + 1) * blk])
    return new


def _perm_heuristic(num_nodes, counts):
    """rank_perm_heuristic (rank_permutation.c:12-87), literally; its qsort on value taken as a
    stable sort (glibc's merge-sort qsort)."""
    org = [dict(value=counts[i], key=i, color=i) for i in range(num_nodes)]
    num_colors = num_nodes
    flag = True
    while flag:
        arr = [dict(value=0, key=i) for i in range(num_colors)]
        for o in org:
            arr[o['color']]['value'] += o['value']
        if num_colors % 2:
            arr[0]['value'] = 0
        arr = sorted(arr, key=lambda a: a['value'])
        org2 = []
        if num_colors % 2 == 0:
            for i in range(num_colors):
                for o in org:
                    if i % 2:
                        if arr[num_colors - 1 - i // 2]['key'] == o['color']:
                            org2.append(dict(o, color=i // 2))
                    else:
                        if arr[i // 2]['key'] == o['color']:
                            org2.append(dict(o, color=i // 2))
        else:
            for o in org:
                if o['color'] == 0:
                    org2.append(dict(o))
            for i in range(num_colors - 1):
                for o in org:
                    if i % 2:
                        if arr[num_colors - 1 - i // 2]['key'] == o['color']:
                            org2.append(dict(o, color=i // 2 + 1))
                    else:
                        if arr[i // 2 + 1]['key'] == o['color']:
                            org2.append(dict(o, color=i // 2 + 1))
        org = org2
        num_colors = (num_colors + 1) // 2
        flag = num_colors > 1
    return [o['key'] for o in org]


def _task_order(N, count, ports):
    """The task order the reference runs with (rank_permutation.c:89-160): its forward pass tests
    its own NULL local rank_perm (:90,106) and so replaces ext_mpi_rank_order's RANK_PERM --
    identity for equal line sizes, else the heuristic over them; the line sizes are count / N
    (remainder to the low nodes), or the whole message in line 0 without reduce-scatter ports
    (allreduce_short, ext_mpi_native.c:667,768-788)."""
    rs = any(p < 0 for p in ports)
    sizes = [count // N + (i < count % N) if rs else (count if i == 0 else 0) for i in range(N)]
    return list(range(N)) if len(set(sizes)) == 1 else _perm_heuristic(N, sizes)


def _allreduce_core_literal(partials, ports):
    """Independent statement of the inter-node algorithm for the oracle's check: the line tables
    of allreduce_core (allreduce_recursive.c:222-453) built as the reference builds them --
    recvfrom node/line per slot, the reducefrom list of the output slot, for the reduce-scatter
    steps (:248-347), the allgather steps that still reduce (:348-403) and the copying ones
    (:404-437) -- and replayed the way raw_code.c:221-356 executes a block: a received line is
    copied into its slot, then the output slot accumulates its reducefrom slots in list order.
    Tasks are the nodes in the order _task_order gives, lines laid out in task order with node
    ranks[k]'s size (ext_mpi_native.c:768-786, rank_permutation.c). Returns the result of every
    node (the tasks of a block may disagree when the allgather steps reduce)."""
    N, count = len(partials), partials[0].size
    rs = [p for p in ports if p < 0]
    ag = [p + 1 for p in ports if p > 0]
    ranks = _task_order(N, count, ports)  # task -> node
    lb = 1
    for p in ag:
        lb *= p
    assert lb == N
    sizes = [count // N + (ranks[k] < count % N) for k in range(N)]
    lo = np.concatenate([[0], np.cumsum(sizes)]).astype(int)
    line = lambda arr, l: arr[lo[l]:lo[l + 1]]  # noqa: E731
    # slots[t][n] = task t's data in slot n (lines n mod lb), block 0: the own partial in 0..lb-1
    slots = [{n: line(partials[ranks[t]], n).copy() for n in range(lb)} for t in range(N)]

    def run_block(recv, red, held):
        new = [dict(x) for x in slots]
        for t in range(N):
            for n, (q, ln) in recv[t].items():
                new[t][n] = held(q, ln).copy()
        for t in range(N):
            for n, lst in red[t].items():
                acc = new[t][n].copy()
                for r in lst:
                    acc = acc + new[t][r]
                new[t][n] = acc
        return new

    gbstep = lb
    for step, port in enumerate(rs):
        p = abs(port)
        last = step == len(rs) - 1
        gnext = gbstep // (p + 1)
        recv, red = [dict() for _ in range(N)], [dict() for _ in range(N)]
        for t in range(N):
            for ln in range(t // gbstep * gbstep, t // gbstep * gbstep + gbstep):
                if ln // gnext == t // gnext:
                    src = lambda i: (t + gnext * (i + 1)) % gbstep + t // gbstep * gbstep  # noqa: E731
                    if not last:
                        base = 3 if step > 0 else 2
                        for i in range(p):
                            recv[t][ln + (base + i) * lb] = (src(i), ln)
                        red[t][ln + 2 * lb] = ([ln + (3 + i) * lb for i in range(p)] if step > 0 else
                                               [ln] + [ln + (2 + i) * lb for i in range(1, p)])
                    else:
                        recv[t][ln + lb] = (src(p - 1), ln)
                        for i in range(p - 1):
                            recv[t][ln + (3 + i) * lb] = (src(i), ln)
                        red[t][ln + lb] = ([ln + (2 + i) * lb for i in range(p)] if step > 0 else
                                           [ln] + [ln + (2 + i) * lb for i in range(1, p)])
        # the sender's copy of line `ln`: its accumulator slot of the previous block
        slots = run_block(recv, red, lambda q, ln: slots[q][ln + 2 * lb] if step > 0 else slots[q][ln])
        gbstep = gnext
    middle, step, g = gbstep, len(rs), 1
    for a in ag:
        gnext = g * a
        recv, red = [dict() for _ in range(N)], [dict() for _ in range(N)]
        for t in range(N):
            if g < middle:  # the allgather steps that reduce (:348-403)
                for ln in range(t // middle * middle, t // middle * middle + middle):
                    for i in range(a - 1):
                        peer = (t + g * (i + 1)) % gnext + t // gnext * gnext
                        recv[t][ln + ((i + 1) if step == 0 else (i + 2)) * lb] = (peer, ln)
                    red[t][ln + lb] = ([ln] + [ln + (i + 1) * lb for i in range(1, a - 1)] if step == 0 else
                                       [ln + (i + 2) * lb for i in range(a - 1)])
            else:  # the copying ones (:404-437)
                for ln in range(t // gnext * gnext, t // gnext * gnext + gnext):
                    if ln // g != t // g:
                        if ln // g > t // g:
                            i = (gnext + ln // g - t // g - 1) % gnext
                        else:
                            i = (gnext + ln // g - t // g) % gnext - 1
                        recv[t][ln + lb] = ((t + g * (i + 1)) % gnext + t // gnext * gnext, ln)
        if g < middle and step == 0:  # the first step of all sends the own partial (slot ln)
            held = lambda q, ln: slots[q][ln]  # noqa: E731
        else:
            held = lambda q, ln: slots[q][ln + lb]  # noqa: E731
        slots = run_block(recv, red, held)
        g, step = gnext, step + 1
    out = []
    for n in range(N):  # node n = task ranks.index(n)
        t = ranks.index(n)
        out.append(np.concatenate([slots[t][k + lb] for k in range(N)]))
    return out


@pytest.mark.parametrize("nodes,ports", [(2, [-1, 1]), (4, [-1, -1, 1, 1]), (3, [-2, 2]), (4, [-3, 3]),
                                         (6, [-1, -2, 2, 1]), (6, [-2, -1, 1, 2]), (8, [-3, -1, 1, 3]),
                                         (9, [-2, -2, 2, 2]), (8, [-1, -1, -1, 1, 1, 1]), (5, [-4, 4]),
                                         # allgather steps that reduce (README: 4(3), 4(-1 1 1), 4(1 1))
                                         (4, [3]), (4, [-1, 1, 1]), (4, [1, 1]), (3, [2]), (6, [-1, 2, 1]),
                                         (8, [-1, 3, 1]), (6, [2, 1]), (2, [1]),
                                         # radix-2 reduce-scatter steps, other allgather radices
                                         (4, [-1, -1, 3]), (8, [-1, -1, -1, 3, 1])])
def test_node_ports_against_literal_line_tables(oracle, nodes, ports):
    """The oracle's inter-node restatement (ref_emulate_node_ports) against an independent,
    literal replay of allreduce_core's line tables: bitwise for float (association observable)."""
    rng = np.random.default_rng(nodes * 31 + len(ports))
    for count in (1, 7, 1000 + nodes, 4099):
        sends = [((rng.random(count) * 2 - 1) * 10.0 ** rng.integers(-4, 5, count)).astype(np.float32)
                 for _ in range(nodes)]
        want = _allreduce_core_literal(sends, ports)
        got = oracle.allreduce_nodes(sends, "6;1 -1 1", nodes, ports=ports)
        for n, out in enumerate(got):
            assert np.array_equal(out, want[n]), (nodes, ports, count, n)
    if nodes == 3:  # the association differs per line: observable, so pinned by the statement
        s = [np.float32([1e8]), np.float32([1.0]), np.float32([-1e8])]
        assert oracle.allreduce_nodes(s, "6;1 -1 1", 3, ports=ports)[0][0] == _allreduce_core_literal(s, ports)[0][0]


def _level_copyin(radices):
    return "6;1 " + " ".join(f"-{r}" for r in radices) + " " + " ".join(str(r) for r in reversed(radices))


def _nest_statement(oracle, data, levels):
    """Sum under the sub-split nest `levels` (radix chains, one per level) of the inputs `data`
    at the positions of one reduce_copies_one_socket call (reduce_copyin.c:970-1084): the level
    folds the members {i g + j} (ranks_loc, :976-981; g = positions / members) with the
    single-level schedule of its radices -- a single-level Allreduce whose own rank order puts
    member q at node rank perm[q] -- and the rest of the nest runs, without a further rank
    order, over the positions {c g + i} (ranks_loci, :1003-1007) on chunk c of the group sums."""
    m = int(np.prod(levels[0]))
    g = len(data) // m
    perm = _rank_order(m, [-r for r in levels[0]], list(range(m)))
    blocks = []
    for j in range(g):
        arr = [None] * m
        for q in range(m):
            arr[perm[q]] = data[q * g + j]
        blocks.append(oracle.allreduce(arr, _level_copyin(levels[0]))[0])
    if len(levels) == 1:
        return blocks[0]
    count = len(data[0])
    lo = np.concatenate([[0], np.cumsum([count // m + (c < count % m) for c in range(m)])]).astype(int)
    return np.concatenate([_nest_statement(oracle, [b[lo[c]:lo[c + 1]] for b in blocks], levels[1:])
                           if lo[c + 1] > lo[c] else blocks[0][:0] for c in range(m)])


@pytest.mark.parametrize("levels", [((4,), (2,)), ((2,), (4,)), ((3,), (2,)), ((2,), (3,)), ((2,), (2,)),
                                    ((4,), (3,)), ((3,), (4,)), ((4,), (4,)), ((2,), (2,), (2,)),
                                    ((2,), (3,), (2,)), ((4,), (2,), (2,)), ((2,), (2,), (4,)),
                                    ((2, 2), (2,)), ((3,), (2, 2)), ((4,), (2, 2)), ((2, 2), (4,)),
                                    ((3, 2), (2,)), ((2, 3), (2, 2)), ((2, 2), (2,), (2,))])
def test_subsplit_fold_order_independent_statement(oracle, levels):
    """Independent statement of a sub-split nest "6;1 <level 0> 1 <members> 1 <level 1> ..." from
    reduce_copies_one_socket (reduce_copyin.c:970-1084), composed of single-level Allreduces
    (themselves pinned by the reference's printed schedules). The node's positions are
    ext_mpi_rank_order over level 0's radices (:1495-1504), identity for one radix (:383-393);
    level 0 folds over the positions {i g + j}, member i ending with chunk i of that group's sum
    (ext_mpi_sizes_displs over the members); the next level folds, over the positions {c g + i}
    -- member c of every group -- chunk c of those group sums, and so on. Bitwise for float and
    double."""
    R = int(np.prod([np.prod(lv) for lv in levels]))
    parts = [" ".join(f"-{r}" for r in lv) + " " + " ".join(str(r) for r in reversed(lv)) for lv in levels]
    copyin = "6;1 " + "".join(f"{p} 1 {int(np.prod(lv))} 1 " for p, lv in zip(parts[:-1], levels[:-1])) + parts[-1]
    pos = _rank_order(R, [-r for r in levels[0]], list(range(R)))
    rng = np.random.default_rng(R * 7 + len(levels))
    for dt in (np.float32, np.float64):
        for count in (1, 7, 1000 + R, 4099):
            sends = [((rng.random(count) * 2 - 1) * 10.0 ** rng.integers(-4, 5, count)).astype(dt) for _ in range(R)]
            want = _nest_statement(oracle, [sends[pos[q]] for q in range(R)], levels)
            for out in oracle.allreduce(sends, copyin):
                assert np.array_equal(out, want), (copyin, dt, count)
