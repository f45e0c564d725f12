"""Host model of k_envq's map-ring protocol (pgtg_amd/csrc/pgtg_env.hip: k_envq, k_qfill), checked
without a GPU: the same arithmetic as the kernel, on random reset patterns.

* Rings of two entries: a reset in launch t takes the head slot and requests the map of spawn
  counter k0 + 10 into it; the helpers serve every request of launch t in launch t + 1.  The entry an
  env takes must always carry the tag of its episode (the kernel reports a mismatch as an error).
* One-round launches: a workgroup lists at most 64 requests; the rest go to the overflow list of its
  residue mod 8, and helper j of a residue serves the overflow items [P_j, P_j + spare_j) (P = the
  prefix sum of the spare lanes 64 - count of the residue's workgroups before it), then items
  tot + (k * nj + j) * 64 ... in whole batches.  Every item must be served exactly once.
"""
import numpy as np

LANES = 64


def _overflow_shares(counts, olen):
    """items served by each helper of one residue: counts = the residue's per-workgroup list lengths"""
    nj = len(counts)
    spare = [LANES - min(c, LANES) for c in counts]
    tot = sum(spare)
    served = [[] for _ in range(nj)]
    pre = 0
    for j in range(nj):
        on = min(olen - pre, spare[j]) if olen > pre else 0
        served[j] += list(range(pre, pre + on))
        pre += spare[j]
        st0 = tot + j * LANES
        while st0 < olen:
            served[j] += list(range(st0, min(st0 + LANES, olen)))
            st0 += nj * LANES
    return served


def test_overflow_items_served_exactly_once():
    rng = np.random.default_rng(3)
    for _ in range(300):
        nj = int(rng.integers(1, 140))
        counts = rng.integers(0, LANES + 1, nj)
        # an overflow list of up to (envs per block - 64) per workgroup (128- and 192-env workgroups)
        olen = int(rng.integers(0, nj * 128 + 1))
        served = _overflow_shares(list(counts), olen)
        flat = sorted(x for s in served for x in s)
        assert flat == list(range(olen)), (nj, olen)


def test_two_entry_rings_always_hold_the_episode():
    """reset patterns from every-step resets to none: the head entry's tag is always the episode's"""
    rng = np.random.default_rng(7)
    n = 500
    for p in (1.0, 0.43, 0.1):
        spawn = np.full(n, 5, np.int64)       # the spawn counter of the next episode
        head = np.zeros(n, np.int64)
        tag = np.zeros((n, 2), np.int64)
        tag[:, 0], tag[:, 1] = spawn, spawn + 5  # k_qfill after the reset
        pending = []                              # requests of the previous launch
        for _t in range(200):
            served, pending = pending, []         # the helpers serve the previous launch's requests
            h0 = head.copy()                      # ring heads at the launch's start
            resets = rng.random(n) < p
            for i in np.nonzero(resets)[0]:
                assert tag[i, h0[i]] == spawn[i], "a taken entry was not made for its episode"
                pending.append((i, h0[i], spawn[i] + 10))
                spawn[i] += 5
                head[i] ^= 1
            for i, slot, k in served:             # written during the launch, visible after it:
                assert not (resets[i] and slot == h0[i]), "a refill raced the take of its slot"
                tag[i, slot] = k


def _envb_launch(rng, p, E, spawn, qn, qh, tag, qcap=LANES):
    """One k_envb launch over one block of E envs (pgtg_env.hip k_envb): the helper refills level 0
    (empty rings, all of them, before any take) and then levels 1, 2 in list order (env order within a
    level) up to qcap entries; a reset takes the head; qn/qh follow the kernel's `have` arithmetic."""
    depth = 3
    F = [[i for i in range(E) if qn[i] <= l] for l in range(depth)]
    for i in F[0]:  # heads of empty rings
        tag[i, qh[i]] = spawn[i]
    served = [(i, l) for l in range(1, depth) for i in F[l]][:qcap]
    for i, l in served:  # written by the helper concurrently with the takes of other slots
        tag[i, (qh[i] + l) % depth] = spawn[i] + 5 * l
    resets = rng.random(E) < p
    for i in range(E):
        have = 1 if qn[i] == 0 else qn[i]
        have += sum(1 for (j, l) in served if j == i)
        if resets[i]:
            assert have >= 1 and tag[i, qh[i]] == spawn[i], "k_envb took an entry not made for its episode"
            # a refill written in this launch never lands on the slot taken (levels >= 1 are other slots)
            assert all(l == 0 or (qh[i] + l) % depth != qh[i] for (j, l) in served if j == i)
            spawn[i] += 5
            qh[i] = (qh[i] + 1) % depth
            have -= 1
        qn[i] = have
    return resets.sum()


def test_three_entry_rings_refilled_per_block():
    """k_envb: capped refills (64 per launch) with deferral through three-entry rings -- every take is
    the episode's map, also when a block resets more envs than its helper refills in one launch"""
    rng = np.random.default_rng(11)
    for E, p in ((128, 0.43), (128, 1.0), (192, 0.6), (16, 0.43), (64, 0.9)):
        spawn = np.full(E, 5, np.int64)
        qn = np.full(E, 3, np.int64)
        qh = np.zeros(E, np.int64)
        tag = np.zeros((E, 3), np.int64)
        for l in range(3):  # k_qfill_b after the reset
            tag[:, l] = spawn + 5 * l
        qcap = 2 * LANES if E > 128 else LANES
        for _t in range(300):
            _envb_launch(rng, p, E, spawn, qn, qh, tag, qcap)
            assert (qn >= 0).all() and (qn <= 3).all()
