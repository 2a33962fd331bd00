"""K1's presence filter (ghostm_amd/csrc/kernels.h k_seed_filter), restated on the
host: the filter may keep more entries than needed (aliased cells), never
fewer. For random per-query entry sets with heavy aliasing (few cells), every
entry that the exact emission rule can use must pass:

  bin b is emitted iff (c(b) > 0 or b = 0) and c(b) + c(b + 1) >= T, so an
  entry in bin x matters iff x <= 1, another entry shares x, or x - 1 or x + 1
  holds an entry.

Stage 1 is the kernel's bitmap (two bits per cell, cell = x mod FSLOTS, the
three cells x - 1, x, x + 1 read from the words holding x - 1 and x + 1, with
wrap-around). Stage 2 (GHOSTM_K1_STAGE2) re-tests the queued entries on a
bitmap built from them alone, cells by a multiplicative hash. The READ2 variant
reads the word pair (w, w + 1) with a guard word mirroring cells 0 and 1. The
GPU parity tests run the kernel itself on the real workloads."""
import random

MASK32 = 0xFFFFFFFF


def needed(bins):
    cnt = {}
    for x in bins:
        cnt[x] = cnt.get(x, 0) + 1
    return [x <= 1 or cnt[x] > 1 or (x - 1) in cnt or (x + 1) in cnt for x in bins]


def stage1(bins, fslots, read2):
    words = [0] * (fslots // 16 + 4)
    for x in bins:  # marks: seen, then twice (the kernel's atomicOr with return)
        cell = x & (fslots - 1)
        sh = (cell & 15) * 2
        old = words[cell >> 4]
        words[cell >> 4] |= 1 << sh
        twice = (old >> sh) & 1
        if twice:
            words[cell >> 4] |= 2 << sh
        if read2 and cell < 2:
            words[fslots // 16] |= (3 if twice else 1) << sh
    keep = []
    for x in bins:
        c0 = (x - 1) & (fslots - 1)
        if read2:
            lo, hi = words[c0 >> 4], words[(c0 >> 4) + 1]
        else:
            c2 = (x + 1) & (fslots - 1)
            lo, hi = words[c0 >> 4], words[c2 >> 4]
        near = (((hi << 32) | lo) >> ((c0 & 15) * 2)) & MASK32
        keep.append(x <= 1 or (near & 0x19) != 0)
    return keep


def stage2(queue, bits):
    cell2 = lambda x: ((x * 2654435761) & MASK32) >> (32 - bits)
    st = {}
    for x in queue:
        c = cell2(x & MASK32)
        st[c] = (st.get(c, 0) | 2) if st.get(c, 0) & 1 else (st.get(c, 0) | 1)
    get = lambda x: st.get(cell2(x & MASK32), 0)
    return [x <= 1 or bool(get(x) & 2) or bool(get(x - 1) & 1) or bool(get(x + 1) & 1) for x in queue]


def test_filter_keeps_every_needed_entry():
    rng = random.Random(11)
    for trial in range(300):
        fslots = rng.choice([64, 256, 1024])
        n = rng.randint(1, 400)
        span = rng.choice([fslots * 4, fslots * 64, 1 << 20])
        bins = [rng.randrange(span) for _ in range(n)]
        # homolog-like runs: the same bin and its neighbours many times
        for _ in range(rng.randint(0, 3)):
            b = rng.randrange(span)
            bins += [b + rng.choice([-1, 0, 0, 0, 1]) for _ in range(rng.randint(2, 40))]
        bins = [max(0, b) for b in bins]
        rng.shuffle(bins)
        need = needed(bins)
        for read2 in (False, True):
            keep = stage1(bins, fslots, read2)
            assert all(k or not nd for k, nd in zip(keep, need)), (trial, read2)
            queue = [x for x, k in zip(bins, keep) if k]
            q_need = needed(queue)
            keep2 = stage2(queue, rng.choice([6, 8, 10]))
            # every entry needed among all entries is queued, and stays needed among the queue
            full_need = dict(zip(range(len(bins)), need))
            qi = [i for i, k in enumerate(keep) if k]
            for j, i in enumerate(qi):
                if full_need[i]:
                    assert q_need[j] and keep2[j], (trial, read2, bins[i])
