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


# ---------------------------------------------------------------------------
# The ring's global slots come from a chunk pool per wave (ipt_hip.hip,
# kPoolChunks / kPoolSlots / kPoolMaxChunks): a lane takes a chunk when its
# pass first writes a chunk's first slot, and a lane that finds the pool empty
# makes its current slot count its ring size for the rest of the path.

POOL_CHUNKS, POOL_SLOTS, POOL_MAX, RING = 63, 16, 4, 63


def lane_passes_pool(K, nl, grant):
    """lane_passes with the pool: grant(j) says whether chunk j can be had
    when the first pass reaches it.  Yields (ulo, uhi, end, ring, mlo,
    chunks held) per sweep; returns the effective ring size via the last."""
    R = min(RING, nl + POOL_MAX * POOL_SLOTS)
    nch = 0
    rhi = 0
    while True:
        rslot, mlo = 0, None
        ring = {}
        k = 0
        while True:
            gs = rslot - nl
            if gs >= 0 and gs % POOL_SLOTS == 0 and gs // POOL_SLOTS >= nch:
                assert rhi == 0 and rslot == k  # only the first pass allocates, before any wrap
                if grant(nch):
                    nch += 1
                else:
                    R, rslot = rslot, 0
            if rslot == 0:
                mlo = k
            assert rslot < nl or (rslot - nl) // POOL_SLOTS < nch  # a global slot lies in a held chunk
            ring[rslot] = k
            rslot = 0 if rslot + 1 == R else rslot + 1
            k += 1
            if k == K or (rhi > 0 and k == rhi):
                break
        if rhi == 0:
            uhi, ulo, end = k, (k - (R if rslot == 0 else rslot)) if k > 0 else 0, True
        else:
            uhi, ulo, end = rhi, rhi - R, False
        yield ulo, uhi, end, [ring.get(i) for i in range(uhi - ulo)], mlo, nch, R
        if ulo <= 0:
            return
        rhi = ulo


@pytest.mark.parametrize("nl", [1, 4, 7, 8])
@pytest.mark.parametrize("fail", [0, 1, 2, 3, None])
@pytest.mark.parametrize("K", list(range(1, 80)) + [130, 200])
def test_pool_limited_ring_tiles_the_path(K, nl, fail):
    chunks = list(lane_passes_pool(K, nl, lambda j: fail is None or j < fail))
    R = chunks[-1][-1]
    full = min(RING, nl + POOL_MAX * POOL_SLOTS)
    reach = nl + (fail if fail is not None else POOL_MAX) * POOL_SLOTS
    assert R == (min(full, reach) if K > min(full, reach) else full)
    cover = []
    for i, (ulo, uhi, end, ring, mlo, nch, _) in enumerate(chunks):
        assert end == (i == 0)
        assert 0 < uhi - ulo <= R and ulo % R == 0
        assert mlo == ulo
        assert ring == list(range(ulo, uhi))
        assert nch <= POOL_MAX and nl + nch * POOL_SLOTS >= min(R, K)
        cover.extend(range(uhi - 1, ulo - 1, -1))
    assert cover == list(range(K - 1, -1, -1))


@pytest.mark.parametrize("chunks,nl", [(POOL_CHUNKS, 4), (POOL_CHUNKS, 7), (6, 7)])
def test_wave_pool_hands_out_each_chunk_once(chunks, nl):
    """64 lanes of one wave tracing Russian-roulette paths one vertex per
    iteration (first passes and replays), with the kernel's hand-out in lane
    order and release after a path's last sweep: no chunk is ever held by two
    lanes, and every chunk is back in the pool at the end."""
    import random
    rnd = random.Random(7)
    free = set(range(chunks))
    owner = {}
    peak = 0
    lanes = [None] * 64
    started, done, dry = 0, 0, 0
    for it in range(20000):
        want = []
        for l in range(64):
            if lanes[l] is None and it < 15000:  # refill
                K = 1
                while rnd.random() < 0.8 and K < 150:
                    K += 1
                lanes[l] = {"K": K, "k": 0, "rslot": 0, "R": min(RING, nl + POOL_MAX * POOL_SLOTS),
                            "held": [], "rhi": 0}
                started += 1
            st = lanes[l]
            if st is None:
                continue
            gs = st["rslot"] - nl
            if gs >= 0 and gs % POOL_SLOTS == 0 and gs // POOL_SLOTS >= len(st["held"]):
                want.append(l)
        for l in want:  # wave-uniform hand-out, lane order
            st = lanes[l]
            if free:
                c = min(free)
                free.remove(c)
                assert c not in owner
                owner[c] = l
                st["held"].append(c)
                peak = max(peak, len(owner))
            else:
                st["R"], st["rslot"] = st["rslot"], 0
                dry += 1
        for l in range(64):
            st = lanes[l]
            if st is None:
                continue
            st["rslot"] = 0 if st["rslot"] + 1 == st["R"] else st["rslot"] + 1
            st["k"] += 1
            if st["k"] == st["K"] or (st["rhi"] > 0 and st["k"] == st["rhi"]):
                K, R, rslot = st["k"], st["R"], st["rslot"]
                ulo = (K - (R if rslot == 0 else rslot)) if st["rhi"] == 0 else st["rhi"] - R
                if ulo > 0:  # replay to ulo, chunks kept
                    st.update(k=0, rslot=0, rhi=ulo)
                else:  # swept to vertex 0: chunks back
                    for c in st["held"]:
                        assert owner.pop(c) == l
                        free.add(c)
                    lanes[l] = None
                    done += 1
    assert all(s is None for s in lanes) and done == started
    assert free == set(range(chunks)) and not owner
    if chunks < POOL_CHUNKS:
        assert dry > 0  # a small pool runs dry: those paths take the shorter ring
    else:
        assert peak < chunks  # q = 0.8 (longer than the scenes' paths): 63 chunks never run out


# ---------------------------------------------------------------------------
# The sub-chunked sweep (ipt_hip.hip, IPT_ADJU_SUB = G): each chunk is swept G
# vertices at a time from its end, one sub-chunk per loop iteration, the lane
# idle meanwhile (its k, rslot, rhi and ring size untouched, so the chunk's
# bounds are recomputed as at its finish); the first M of a sub-chunk comes
# from the per-lane array the pass fills at every ring slot that is a multiple
# of G (k > 0; vertex 0's M is 1).

def lane_sweeps_sub(K, nl, grant, G):
    """Per sweep: (slo, uhi, end, ring slots of [slo, uhi), M capture of
    slo or 'one', iteration).  Follows the kernel's state machine."""
    R = min(RING, nl + POOL_MAX * POOL_SLOTS)
    nch, rhi, it = 0, 0, 0
    mring = {}
    while True:
        rslot, ring, k = 0, {}, 0
        while True:  # one pass
            gs = rslot - nl
            if gs >= 0 and gs % POOL_SLOTS == 0 and gs // POOL_SLOTS >= nch:
                if grant(nch):
                    nch += 1
                else:
                    R, rslot = rslot, 0
            if rslot % G == 0 and k > 0:
                mring[rslot // G] = k  # M before vertex k's update
            ring[rslot] = k
            rslot = 0 if rslot + 1 == R else rslot + 1
            k += 1
            it += 1
            if k == K or (rhi > 0 and k == rhi):
                break
        usub, first = 0, True
        while True:  # the finish, then one sub-chunk per iteration
            uhi = usub if usub else (k if rhi == 0 else rhi)
            ulo = (k - (R if rslot == 0 else rslot)) if rhi == 0 else rhi - R
            slo = ulo + G * ((uhi - 1 - ulo) // G)
            m = "one" if slo == 0 else mring.get((slo - ulo) // G)
            yield slo, uhi, first and rhi == 0, [ring.get(slo - ulo + i) for i in range(uhi - slo)], m, it
            first = False
            if slo > ulo:
                usub = slo
                it += 1  # the next sub-chunk in the next iteration
                continue
            break
        if ulo <= 0:
            return
        rhi = ulo


@pytest.mark.parametrize("G", [4, 8, 16])
@pytest.mark.parametrize("nl", [1, 6, 8])
@pytest.mark.parametrize("fail", [0, 2, None])
@pytest.mark.parametrize("K", list(range(1, 40)) + list(range(40, 80, 3)) + [130, 200])
def test_sub_chunked_sweep_tiles_the_path(K, nl, fail, G):
    sweeps = list(lane_sweeps_sub(K, nl, lambda j: fail is None or j < fail, G))
    cover = []
    for i, (slo, uhi, end, ring, m, _) in enumerate(sweeps):
        assert end == (i == 0)                     # only the path's last sub-chunk carries the escape terms
        assert 0 < uhi - slo <= G                  # a round's chain: at most G - 1 steps
        assert ring == list(range(slo, uhi))       # task kk reads ring slot slo - ulo + kk
        assert m == ("one" if slo == 0 else slo)   # the sub-chunk's first M: the pass's capture at slo
        cover.extend(range(uhi - 1, slo - 1, -1))
    assert cover == list(range(K - 1, -1, -1))     # every vertex once, last to first
    its = [s[-1] for s in sweeps]
    assert its == sorted(its)
