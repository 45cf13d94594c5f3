"""Generate tests/golden/kat_*.npz: the reference's own known-answer test, restated.

src/mpi/debug_persistent.c:491-497 fills every rank's send buffer, viewed as `long` words, with
    word[i] = world_rank * count + i + 73          (host buffers; :426-432 uses +0 on the GPU)
and, when the byte count is not a multiple of 8, sets the last int to world_rank*count+count-1.
It then runs the schedule with MPI_LONG (8-byte types) or MPI_INT (4-byte types) and compares
word-for-word with PMPI_Allreduce (:507-545). Integer sums are order-independent, so the
expected output is the plain element-wise sum over ranks, computed here with numpy int64
arithmetic (independent of the oracle). Run: python tests/golden/make_kat_fixtures.py
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def kat_input(count, itemsize, world_rank, add):
    nbytes = count * itemsize
    words = np.arange(nbytes // 8, dtype=np.int64) + world_rank * count + add
    raw = np.zeros(nbytes, dtype=np.uint8)
    raw[: words.size * 8] = words.view(np.uint8)
    if nbytes % 8:
        raw[(count - 1) * 4:count * 4] = np.array([world_rank * count + count - 1], dtype=np.int32).view(np.uint8)
    return raw.view(np.int32 if itemsize == 4 else np.int64)


def main():
    cases = []
    for R in (2, 4, 8):
        for count, itemsize in ((1001, 4), (1000, 4), (777, 8), (4096, 8)):
            for add in (73, 0):
                cases.append((R, count, itemsize, add))
    for R, count, itemsize, add in cases:
        ins = np.stack([kat_input(count, itemsize, r, add) for r in range(R)])
        expected = ins.astype(np.int64).sum(axis=0).astype(ins.dtype)
        name = f"kat_R{R}_n{count}_t{itemsize}_a{add}.npz"
        np.savez_compressed(os.path.join(HERE, name), inputs=ins, expected=expected,
                            meta=np.array([R, count, itemsize, add], dtype=np.int64))
    print(f"wrote {len(cases)} fixtures")


if __name__ == "__main__":
    main()
