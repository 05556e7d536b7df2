"""The compaction-merge oracle (ora_merge_kvs, CompactAndMergeKVs merge.go:42-94;
SURVEY.md §8(f) f2) against the reference's own test and an independent
Python restatement of container/heap + the merge loop.

Tie order: the reference pushes into Go's container/heap, which is not
stable.  ORA_TIE_GOHEAP replays that heap exactly; ORA_TIE_INPUT pops equal
keys in input order, the contract merge.go:41 states ("keep the newest pair,
the newest comes first").  test_goheap_tie_order_differs records how often
the two disagree on compaction-shaped inputs -- the reason the GPU path
implements the stated contract.
"""
import random
from itertools import groupby

import numpy as np
import pytest

import pyoracle as ora

T = ora.merge_pairs.__globals__["TIE_INPUT"], ora.merge_pairs.__globals__["TIE_GOHEAP"]
TOMB = "～DELETED～".encode()


def goheap_order(keys):
    """container/heap Push x n then Pop x n (Go's heap.go up/down), Less = <."""
    h = []

    def up(j):
        while j > 0:
            i = (j - 1) // 2
            if not keys[h[j]] < keys[h[i]]:
                break
            h[i], h[j] = h[j], h[i]
            j = i

    def down(i, n):
        while True:
            j1 = 2 * i + 1
            if j1 >= n:
                break
            j = j1
            if j1 + 1 < n and keys[h[j1 + 1]] < keys[h[j1]]:
                j = j1 + 1
            if not keys[h[j]] < keys[h[i]]:
                break
            h[i], h[j] = h[j], h[i]
            i = j

    for x in range(len(keys)):
        h.append(x)
        up(len(h) - 1)
    out = []
    while h:
        n = len(h) - 1
        h[0], h[n] = h[n], h[0]
        down(0, n)
        out.append(h.pop())
    return out


def merge_loop(pairs, order, level, threshold):
    """merge.go:57-91 over a pop order -> (written indices, file starts)."""
    out, starts, size, last = [], [0], 0, b""
    for p in order:
        k, v = pairs[p]
        if len(last) > 0 and k == last:
            continue
        if v != TOMB or level < 6:
            out.append(p)
            size += 4 + len(k) + 4 + len(v) + 8
            last = k
        if size >= threshold:
            starts.append(len(out))
            size, last = 0, b""
    if size > 0:
        starts.append(len(out))
    return out, starts


def model(pairs, level, threshold, tie):
    keys = [k for k, _ in pairs]
    order = (goheap_order(keys) if tie == T[1]
             else sorted(range(len(pairs)), key=lambda i: (keys[i], i)))
    return merge_loop(pairs, order, level, threshold)


def random_pairs(rng, n, alphabet=b"ab\x00z", maxlen=12, tomb=0.2):
    pairs = []
    for _ in range(n):
        k = bytes(rng.choice(alphabet) for _ in range(rng.randint(0, maxlen)))
        v = TOMB if rng.random() < tomb else bytes(rng.randint(97, 122) for _ in range(rng.randint(0, 30)))
        pairs.append((k, v))
    return pairs


def test_reference_merge_test_vector():
    """merge_test.go:12-60: 4 entries, the first "beta" (B) wins."""
    pairs = [(b"alpha", b"A"), (b"beta", b"B"), (b"beta", b"B2"), (b"carrot", b"C"), (b"delta", b"D")]
    for tie in T:
        out, starts = ora.merge_pairs(pairs, 1, 2 * 1024 * 1024, tie)
        assert [pairs[i] for i in out] == [(b"alpha", b"A"), (b"beta", b"B"), (b"carrot", b"C"),
                                           (b"delta", b"D")]
        assert list(starts) == [0, 4]


@pytest.mark.parametrize("tie", [0, 1])
def test_oracle_vs_python_model(tie):
    rng = random.Random(5 + tie)
    for trial in range(300):
        pairs = random_pairs(rng, rng.randint(0, 60))
        level = rng.choice([1, 5, 6])
        threshold = rng.choice([1, 40, 100, 400, 1 << 21])
        out, starts = ora.merge_pairs(pairs, level, threshold, tie)
        want_out, want_starts = model(pairs, level, threshold, tie)
        assert list(out) == want_out and list(starts) == want_starts, (trial, level, threshold)


def test_unique_keys_make_tie_order_irrelevant():
    rng = random.Random(8)
    for _ in range(100):
        keys = sorted({bytes(rng.randint(0, 255) for _ in range(rng.randint(0, 10)))
                       for _ in range(rng.randint(0, 80))})
        rng.shuffle(keys)
        pairs = [(k, TOMB if rng.random() < 0.2 else b"v") for k in keys]
        for level in (1, 6):
            a = ora.merge_pairs(pairs, level, 64, T[0])
            b = ora.merge_pairs(pairs, level, 64, T[1])
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_flush_inside_a_group_writes_the_next_duplicate():
    """merge.go:80-84 resets lastWrittenKey at a flush: a duplicate right
    after the flush is written again, into the next file."""
    pairs = [(b"k", b"new" * 10), (b"k", b"old"), (b"m", b"x")]
    out, starts = ora.merge_pairs(pairs, 1, 40, T[0])  # first pair alone reaches 40
    assert list(out) == [0, 1, 2] and list(starts) == [0, 1, 3]


def test_level6_tombstone_uncovers_an_older_value():
    """At level 6 a tombstone is not written and lastWrittenKey keeps the
    previous key, so the next (older) pair of the same key is written."""
    pairs = [(b"k", TOMB), (b"k", b"old"), (b"j", b"1")]
    out, _ = ora.merge_pairs(pairs, 6, 1 << 21, T[0])
    assert list(out) == [2, 1]
    out, _ = ora.merge_pairs(pairs, 5, 1 << 21, T[0])
    assert list(out) == [2, 0]


def test_empty_keys_are_never_deduplicated():
    pairs = [(b"", b"a"), (b"", b"b"), (b"x", b"c"), (b"x", b"d")]
    out, _ = ora.merge_pairs(pairs, 1, 1 << 21, T[0])
    assert list(out) == [0, 1, 2]


def test_goheap_tie_order_differs():
    """The reference's heap does not keep input order among equal keys: on
    concatenated sorted runs (loadLevelData's shape) a sizeable share of the
    duplicate groups keep a different pair than the input-order contract."""
    rng = random.Random(3)
    differ = groups = 0
    for _ in range(200):
        pairs = []
        for r in range(rng.randint(2, 5)):
            ks = sorted(rng.sample(range(300), rng.randint(10, 60)))
            pairs += [(b"key%04d" % k, b"run%d" % r) for k in ks]
        a, _ = ora.merge_pairs(pairs, 1, 1 << 21, T[0])
        b, _ = ora.merge_pairs(pairs, 1, 1 << 21, T[1])
        groups += len(a)
        differ += int(np.sum(a != b))
    assert 0.02 < differ / groups < 0.5


def test_goheap_winner_depends_on_larger_keys_pushed_later():
    """Evidence for DESIGN.md §3 (f2 tie rule): under the reference's heap
    (merge.go:45-80, container/heap up/down) the pair kept for key k15 changes
    when only pairs with LARGER keys are appended after the group.  The winner
    is therefore not a function of the group's own members and input
    positions: any exact method must replay the heap's whole push/pop history
    (a sequential O(n log n) chain), which is why the GPU merge implements
    the stated input-order contract (merge.go:41, merge_test.go:25,53)."""
    pre = [(b"k24", b"x0"), (b"k14", b"x1"), (b"k30", b"x2")]
    group = [(b"k15", b"A"), (b"k15", b"B")]
    ext = [(b"k24", b"y"), (b"k19", b"y"), (b"k21", b"y"), (b"k19", b"y")]

    def kept(pairs, tie):
        out, _ = ora.merge_pairs(pairs, 1, 1 << 21, tie)
        return [pairs[i][1] for i in out if pairs[i][0] == b"k15"]

    assert kept(pre + group, T[1]) == [b"B"]
    assert kept(pre + group + ext, T[1]) == [b"A"]
    # the input-order contract keeps the first pair either way
    assert kept(pre + group, T[0]) == kept(pre + group + ext, T[0]) == [b"A"]


def test_library_goheap_pop_order_matches_restatement():
    """lsm_goheap_pop_order_host (the host replay behind LSM_TIE_GOHEAP) is
    container/heap's pop order: against the Python restatement above, over
    dense key ranks, on random keys with many ties and on concatenated
    sorted runs (compaction-shaped)."""
    from lsmgpu import _lib, goheap_pop_order
    lib = _lib.load()
    rng = random.Random(12)
    cases = []
    for _ in range(150):
        cases.append([bytes(rng.choice(b"abc") for _ in range(rng.randint(0, 4)))
                      for _ in range(rng.randint(0, 200))])
    for _ in range(30):
        keys = []
        for r in range(rng.randint(2, 6)):
            keys += [b"key%04d" % k for k in sorted(rng.sample(range(400), rng.randint(5, 90)))]
        cases.append(keys)
    for keys in cases:
        uniq = {k: i for i, k in enumerate(sorted(set(keys)))}
        rank = np.array([uniq[k] for k in keys], np.uint32)
        got = goheap_pop_order(lib, rank)
        assert list(got) == goheap_order(keys)
    # the winner-depends-on-later-keys case, through ranks
    keys = [b"k24", b"k14", b"k30", b"k15", b"k15", b"k24", b"k19", b"k21", b"k19"]
    uniq = {k: i for i, k in enumerate(sorted(set(keys)))}
    assert list(goheap_pop_order(lib, np.array([uniq[k] for k in keys], np.uint32))) == \
        goheap_order(keys)
