"""Pins the oracle's Rest (src/algo/Rest.cpp:31-77) to src/test/rest.cpp
(Rest_main, Rest_self, Rest_of_empty).  CPU only."""
from oracle import oracle as orc


def _lens(blocks):
    return sorted(mx - mn + 1 for b in blocks for _, mn, mx, _, _ in b)


def test_rest_main():
    """rest.cpp:19-55: 5 stretches; by length 1, 1, 5, 8, 15 (the test's
    Filter min-fragment 2 / 6 / 8 / 9 steps keep 3 / 2 / 2 / 1 of them)."""
    src = orc.BlockSetOracle(["tGGtccgagcgGAcggcc", "tGGtccgagcggacggcc"], ["s1", "s2"])
    src.set_blocks([[(0, 1, 2, 1, None), (1, 1, 2, 1, None)], [(0, 11, 12, 1, None)]])
    src.apply("Rest")
    rest = src.blocks()[2:]
    assert len(rest) == 5 and all(len(b) == 1 for b in rest)
    lens = _lens(rest)
    assert lens == [1, 1, 5, 8, 15]
    assert [sum(x >= m for x in lens) for m in (2, 6, 8, 9)] == [3, 2, 2, 1]
    assert sorted((s, mn, mx) for b in rest for s, mn, mx, _, _ in b) == \
        [(0, 0, 0), (0, 3, 10), (0, 13, 17), (1, 0, 0), (1, 3, 17)]


def test_rest_self_and_empty():
    """rest.cpp:57-79: Rest into the same set; a set without blocks."""
    o = orc.BlockSetOracle(["AAA"], ["s1"])
    o.set_blocks([[(0, 1, 1, 1, None)]])
    o.apply("Rest")
    assert len(o.blocks()) == 3
    o = orc.BlockSetOracle(["AAA"], ["s1"])
    o.set_blocks([])
    o.apply("Rest")
    assert o.blocks() == [[(0, 0, 2, 1, None)]]
