"""The unbounded adjoint's chunk protocol (ipt_hip.hip, MODE_ADJU), restated
per lane in Python: a path of K vertices with a ring of R record slots is
swept in chunks [j R, min((j + 1) R, K)) from the last to the first, each
right after the pass (first pass or replay from the camera ray) that wrote
its records into ring slots 0 .. len - 1 and captured its prefix throughput
at its first vertex.  Checks the chunks tile the path exactly once, back to
front, that every chunk's records and Mlo are the ones its pass left in the
ring, and the replay cost (vertex traces beyond the first pass)."""
import pytest


def lane_passes(K, R):
    """Run one lane's state machine; yield (ulo, uhi, end, ring, mlo, traced)
    per sweep, where ring = vertex index per slot and mlo = capture vertex."""
    rhi = 0
    total = 0
    while True:
        rslot, mlo = 0, None
        ring = [None] * R
        k = 0
        while True:  # one pass: vertex k is recorded in slot rslot
            if rslot == 0:
                mlo = k  # Mlo = M before vertex k's update
            ring[rslot] = k
            rslot = 0 if rslot + 1 == R else rslot + 1
            k += 1
            total += 1
            if k == K or (rhi > 0 and k == rhi):
                break
        if rhi == 0:
            uhi, ulo, end = k, (k - (R if rslot == 0 else rslot)) if k > 0 else 0, True
        else:
            uhi, ulo, end = rhi, rhi - R, False
        yield ulo, uhi, end, list(ring), mlo, total
        if ulo <= 0:
            return
        rhi = ulo


@pytest.mark.parametrize("R", [1, 2, 3, 8, 24])
@pytest.mark.parametrize("K", list(range(1, 60)) + [97, 200])
def test_chunks_tile_the_path_back_to_front(K, R):
    chunks = list(lane_passes(K, R))
    cover = []
    for i, (ulo, uhi, end, ring, mlo, _) in enumerate(chunks):
        assert end == (i == 0)                      # only the first sweep ends the path (escape terms)
        assert 0 < uhi - ulo <= R and ulo % R == 0  # ring-aligned, fits the ring
        assert mlo == ulo                           # Mlo captured at the chunk's first vertex
        assert ring[:uhi - ulo] == list(range(ulo, uhi))  # task kk reads slot kk
        cover.extend(range(uhi - 1, ulo - 1, -1))
    assert cover == list(range(K - 1, -1, -1))      # every vertex once, last to first
    # replayed vertex traces: the full chunks before the last one, each replayed from vertex 0
    m = (K - 1) // R
    assert chunks[-1][-1] - K == R * m * (m + 1) // 2
