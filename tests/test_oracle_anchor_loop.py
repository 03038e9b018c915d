"""The oracle's AnchorLoop restatement (oracle/npge_oracle.cpp anchor_loop,
lua_lib.lua:711-737) on CPU: the properties its processors promise.
AddingLoopBySize ("Align and move overlapless from other to target",
TrySmth.cpp:180-182) leaves no two overlapping blocks; ExtendLoop ends on a
fixpoint of its Pipe (a second run changes nothing it would not repeat);
AnchorLoop keeps every block aligned and is deterministic."""
from oracle import oracle as orc
from npge_amd import synth


def overlaps(blocks):
    seen = {}
    for bi, b in enumerate(blocks):
        for f in b:
            seen.setdefault(f[0], []).append((f[1], f[2], bi))
    bad = 0
    for iv in seen.values():
        iv.sort()
        for (a0, a1, ab), (b0, b1, bb) in zip(iv, iv[1:]):
            if b0 <= a1:
                bad += 1
    return bad


def _aligned_anchors(cfg):
    from npge_amd.anchor_loop import anchor_blocks
    names, seqs = synth.genome_set(cfg)
    o = orc.BlockSetOracle(seqs, names)
    o.set_blocks(anchor_blocks(orc.AnchorFinder().run(seqs, names)))
    o.apply("DummyAligner")
    return names, seqs, o


def overlapping_input(cfg="tiny"):
    """The anchors, DummyAligner'd and extended by FragmentsExtender (100 bp a
    side): heavily overlapping blocks, as ExtendLoop hands AddingLoopBySize."""
    from npge_amd.anchor_loop import anchor_blocks
    names, seqs = synth.genome_set(cfg)
    o = orc.BlockSetOracle(seqs, names)
    o.set_blocks(anchor_blocks(orc.AnchorFinder().run(seqs, names)))
    o.apply("DummyAligner")
    o.apply("FragmentsExtender")
    return names, seqs, o.blocks()


def test_adding_loop_by_size_is_overlapless():
    names, seqs, blocks = overlapping_input()
    o = orc.BlockSetOracle(seqs, names)
    o.set_blocks(blocks)
    assert overlaps(blocks) > 0
    o.apply("AddingLoopBySize")
    out = o.blocks()
    assert 0 < len(out) < len(blocks)
    assert overlaps(out) == 0
    before = set(tuple(sorted(f[:4] for f in b)) for b in blocks)
    assert any(tuple(sorted(f[:4] for f in b)) not in before for b in out)  # SmthUnion cut some
    for b in out:
        assert all(f[4] is not None and len(f[4]) == len(b[0][4]) for f in b)


def test_extend_loop_output():
    names, seqs, o = _aligned_anchors("tiny")
    o.apply("ExtendLoop")
    out = o.blocks()
    assert out and overlaps(out) == 0
    assert max(len(b[0][4]) for b in out) > 100  # grown past the 20-mers


def test_anchor_loop_deterministic_and_aligned():
    names, seqs = synth.genome_set("rtiny")
    res = []
    for _ in range(2):
        o = orc.BlockSetOracle(seqs, names)
        o.apply("DraftPangenome")
        o.apply("AnchorLoop")
        res.append((sorted(tuple(sorted(b)) for b in o.blocks()), o.anchor_loop_stats()))
        for b in o.blocks():
            rows = [f[4] for f in b]
            assert all(r is not None and len(r) == len(rows[0]) for r in rows)
    assert res[0] == res[1]
    st = res[0][1]
    assert st["cons_seqs"] > 0 and st["cons_anchors"] > 0 and st["split_blocks"] > 0


def test_anchor_loop_invariants_whatever_the_pinned_choices():
    """Properties of the AnchorLoop result that hold whatever the conventions
    this port pins where the reference is not reproducible (the consensus
    sequences' fresh names, SplitExtendable's std::set<Fragment*> order, the
    sort tie-breaks; DESIGN.md "The AnchorLoop pipe"): every block's rows
    have one length and hold its fragments' letters, the closing Align's
    Filter leaves every block as it is, and every DraftPangenome block the
    pipe started from is still there (on rtiny; the result may overlap
    itself: the consensus blocks DeConSeq maps back are not unioned against
    them)."""
    names, seqs = synth.genome_set("rtiny")
    o = orc.BlockSetOracle(seqs, names)
    o.apply("DraftPangenome")
    draft = {tuple(sorted(f[:4] for f in b)) for b in o.blocks()}
    o.apply("AnchorLoop")
    out = o.blocks()
    assert out
    for b in out:
        rows = [f[4] for f in b]
        assert all(r is not None and len(r) == len(rows[0]) for r in rows)
        for (q, mn, mx, ori, row) in b:
            assert len(row) - row.count("-") == mx - mn + 1
    f2 = orc.BlockSetOracle(seqs, names)
    f2.set_blocks(out)
    f2.apply("Filter")
    assert sorted(tuple(sorted(b)) for b in f2.blocks()) == sorted(tuple(sorted(b)) for b in out)
    assert draft <= {tuple(sorted(f[:4] for f in b)) for b in out}
