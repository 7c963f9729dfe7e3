"""The launches' dynamic work distribution (ipt_hip.hip: launch_inst's chunk
sizes and grab count, chunk_range, the kernel's grab), restated in Python
and run against random interleavings of the waves' atomics:

* every work item of the launch is handed out exactly once (none skipped,
  none traced twice), with fixed chunks and with guided sizes (big chunks,
  then IPT_GUIDED_TAIL / IPT_BF_TAIL small ones per wave: the BVH instances,
  and since round 6 the brute-force ones with IPT_BF_BIG = 2);
* the counter word sees exactly the number of grabs the host computes
  (launch_grabs), so the grab that returns grabs - 1 is the launch's last
  and may zero the word for the next launch on the stream (grab_failed).

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


def host_shape(units, waves, c0, big, tail_per_wave, bvh_guided):
    """launch_inst (non-fused): chunk c, small, big-chunk count nb, grabs."""
    guided = bvh_guided or big > 1
    small = c0
    c = c0 * (big if not bvh_guided else 1)
    tail = waves * tail_per_wave * small if guided else 0
    nb = (units - tail) // c if guided and units > tail else 0
    return guided, c, small, nb, launch_grabs(guided, units, c, small, nb, waves)


def run_launch(units, waves, c0, big=1, tail_per_wave=4, bvh_guided=False, seed=0):
    """Waves take turns at random (one grab or one chunk's work per turn);
    returns (items in hand-out order, grabs seen, host grabs, final word)."""
    guided, c, small, nb, grabs = host_shape(units, waves, c0, big, tail_per_wave, bvh_guided)
    ctr = seen = 0
    out = []
    ranges = [list(chunk_range(guided, w, units, c, small, nb)) for w in range(waves)]  # the waves' own chunks
    rng = random.Random(seed)
    live = list(range(waves))
    while live:
        w = rng.choice(live)
        s, e = ranges[w]
        if s < e:
            out.extend(range(s, e))  # the wave traces its chunk
            ranges[w] = [e, e]
            continue
        g = ctr  # the kernel's grab (atomicAdd, lane 0)
        ctr += 1
        seen += 1
        s, e = chunk_range(guided, waves + g, units, c, small, nb)
        if s < units:
            ranges[w] = [s, e]
        else:
            assert g + 1 <= grabs  # a failed grab: the one returning grabs - 1 zeroes the word
            if g + 1 == grabs:
                ctr = 0
            live.remove(w)
    return out, seen, grabs, ctr


CASES = [
    # (items, waves, c0, big, tail/wave, bvh-guided)
    (16777216 // 64, 6144 // 64, 128, 1, 4, False),  # C2 adjoint shape, scaled down 64x
    (16777216 // 64, 6144 // 64, 128, 2, 4, False),  # ... guided (the shipped IPT_BF_BIG)
    (16777216 // 64, 6144 // 64, 128, 4, 2, False),
    (100000, 40, 64, 1, 4, True),                    # BVH guided
    (4096, 160, 128, 2, 4, False),                   # fewer chunks than waves
    (64, 16, 128, 8, 4, False),
    (24 * 8 * 7 + 5, 8, 64, 2, 3, False),            # ragged last chunk
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_every_item_once_and_grab_count_exact(case, seed):
    n, waves, c0, big, tail, bvh = case
    out, seen, grabs, ctr = run_launch(n, waves, c0, big, tail, bvh, seed)
    assert sorted(out) == list(range(n))
    assert seen == grabs  # exactly the host's count ...
    assert ctr == 0       # ... so the word ends the launch zeroed


def test_guided_brute_force_cuts_grabs():
    """The guided sizes for the brute-force instances (IPT_BF_BIG = 2, the
    shipped value) cut the C2 adjoint's grabs 131 072 -> 77 824 for the same
    tail (4 chunks of 128 items per wave)."""
    n, waves = 16777216, 6144
    g1 = host_shape(n, waves, 128, 1, 4, False)[-1]
    g2 = host_shape(n, waves, 128, 2, 4, False)[-1]
    assert (g1, g2) == (131072, 77824)
