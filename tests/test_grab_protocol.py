"""The launches' dynamic work distribution (ipt_hip.hip: launch_inst's chunk
sizes and grab counts, chunk_range, the kernel's grab loop), restated in
Python and run against a random interleaving of the waves' atomics:

* every work item of the launch is handed out exactly once (none skipped,
  none traced twice) -- guided sizes (big chunks, then IPT_BF_TAIL /
  IPT_GUIDED_TAIL small ones per wave) and XCD bands (items enumerated band
  by band, each band with its own counter, a wave moving on to the next band
  after one failed grab until it has failed on every band);
* every counter word sees exactly the number of grabs the host computes
  (launch_grabs + the bands' extra failed grabs), so the grab that returns
  grabs - 1 is the word's last and may zero it for the next launch on the
  stream (grab_failed);
* the banded item enumeration (item_split) is a permutation of the
  (pixel, sample) pairs, sample-major inside a band.

The GPU side of the same contract: tests/test_gpu.py
test_counter_reset_over_launch_shapes (launches of many shapes back to back
on one stream, each equal to the same launch alone)."""
import random

import pytest


def launch_grabs(guided, units, c, small, nb, rw):  # ipt_hip.hip launch_grabs
    chunks = nb + (units - nb * c + small - 1) // small if guided else (units + c - 1) // c
    return (chunks - rw if chunks > rw else 0) + rw


def chunk_range(guided, g, units, c, small, nb):  # ipt_hip.hip chunk_range
    if not guided or g < nb:
        start, ln = g * c, c
    else:
        start, ln = nb * c + (g - nb) * small, small
    return start, min(start + ln, units)


def host_shape(n_items, waves, c0, big, tail_per_wave, bvh_guided, R):
    """launch_inst (non-fused): chunk c, small, big-chunk count nb and grabs per word."""
    guided = bvh_guided or big > 1
    small = c0
    c = c0 * (big if not bvh_guided else 1)
    rw, ur = waves // R, n_items // R
    tail = rw * tail_per_wave * small if guided else 0
    nb = (ur - tail) // c if guided and ur > tail else 0
    grabs = launch_grabs(guided, ur, c, small, nb, rw) + (R - 1) * rw
    return guided, c, small, nb, rw, ur, grabs


def run_launch(n_items, waves, c0, big=1, tail_per_wave=4, bvh_guided=False, R=1, seed=0):
    """Waves take turns at random (one grab or one chunk's work per turn);
    returns (items handed out in order of hand-out, grabs seen per word, host grabs)."""
    guided, c, small, nb, rw, ur, grabs = host_shape(n_items, waves, c0, big, tail_per_wave, bvh_guided, R)
    ctr = [0] * R
    seen = [0] * R
    out = []
    state = []
    for w in range(waves):
        band = w % R if R > 1 else 0  # block b starts on band b % R (waves of a block: same band)
        wave_in_band = w // R
        s, e = chunk_range(guided, wave_in_band, ur, c, small, nb)
        state.append({"band": band, "tried": 0, "next": band * ur + s, "end": band * ur + e, "done": False})
    rng = random.Random(seed)
    live = list(range(waves))
    while live:
        w = rng.choice(live)
        st = state[w]
        if st["next"] < st["end"]:
            out.extend(range(st["next"], st["end"]))  # the wave traces its chunk
            st["next"] = st["end"]
            continue
        b = st["band"]  # the kernel's grab loop (one grab per turn)
        g = ctr[b]
        ctr[b] += 1
        seen[b] += 1
        s, e = chunk_range(guided, rw + g, ur, c, small, nb)
        if s < ur:
            st["next"], st["end"] = b * ur + s, b * ur + e
        else:
            assert g + 1 <= grabs  # a failed grab: the one returning grabs - 1 zeroes the word
            if g + 1 == grabs:
                ctr[b] = 0
            st["tried"] += 1
            st["band"] = 0 if b + 1 == R else b + 1
            if st["tried"] >= R:
                live.remove(w)
    return out, seen, grabs, ctr


CASES = [
    # (items, waves, c0, big, tail/wave, bvh-guided, bands)
    (16777216 // 64, 6144 // 64, 128, 1, 4, False, 1),   # C2 adjoint shape, scaled down 64x
    (16777216 // 64, 6144 // 64, 128, 4, 4, False, 1),
    (16777216 // 64, 6144 // 64, 128, 1, 4, False, 8),
    (16777216 // 64, 6144 // 64, 128, 4, 2, False, 8),
    (100000, 40, 64, 1, 4, True, 1),                    # BVH guided
    (100000, 40, 64, 1, 4, True, 4),
    (4096, 160, 128, 4, 4, False, 8),                   # fewer chunks than waves
    (64, 16, 128, 8, 4, False, 2),
    (24 * 8 * 7, 8, 64, 2, 3, False, 8),                # ragged last chunks per band
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_every_item_once_and_grab_counts_exact(case, seed):
    n, waves, c0, big, tail, bvh, R = case
    assert n % R == 0 and waves % R == 0  # band_count's conditions (npix % R, grid % R)
    out, seen, grabs, ctr = run_launch(n, waves, c0, big, tail, bvh, R, seed)
    assert sorted(out) == list(range(n))
    assert seen == [grabs] * R       # each word: exactly the host's count
    assert ctr == [0] * R            # ... so every word ends the launch zeroed


def test_guided_brute_force_cuts_grabs():
    """The guided sizes for the brute-force instances (IPT_BF_BIG = 2, the
    shipped value) cut the C2 adjoint's grabs 131 072 -> 77 824 for the same
    tail (4 chunks of 128 items per wave)."""
    n, waves = 16777216, 6144
    g1 = host_shape(n, waves, 128, 1, 4, False, 1)[-1]
    g2 = host_shape(n, waves, 128, 2, 4, False, 1)[-1]
    g4 = host_shape(n, waves, 128, 4, 4, False, 1)[-1]
    assert (g1, g2) == (131072, 77824)
    assert g4 < 0.45 * g1


def banded_item_split(w, npix, spp, R):  # ipt_hip.hip item_split, nband > 1
    bnpix = npix // R
    band_items = bnpix * spp
    b = w // band_items
    wb = w - b * band_items
    q = wb // bnpix
    return b * bnpix + (wb - q * bnpix), q


@pytest.mark.parametrize("npix,spp,R", [(64, 4, 8), (512 * 8, 3, 8), (96, 5, 4), (16, 1, 2)])
def test_banded_enumeration_is_a_permutation(npix, spp, R):
    pairs = [banded_item_split(w, npix, spp, R) for w in range(npix * spp)]
    assert sorted(pairs) == [(lp, s) for lp in range(npix) for s in range(spp)]
    # sample-major inside a band: consecutive items of a band are consecutive pixels
    bn = npix // R
    for w in range(npix * spp - 1):
        (l0, s0), (l1, s1) = pairs[w], pairs[w + 1]
        if (w + 1) % bn:
            assert (l1, s1) == (l0 + 1, s0)
