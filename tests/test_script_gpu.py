"""The golden fixtures through the fixed-form script runner (npge_amd/script.py),
the way meta_test.cxx:53-102 runs test-script/*/script.npge: --in-blocks
in.fasta, the script's processors (HIP library behind the Processor mirror),
the written block set compared with out.fasta by blockset_hash.  The scripts
below restate each case's processor sequence and options in the runner's
grammar (run_main / run calls, a for loop, BlockSet.new and table calls)."""
import os

import pytest

from npge_amd import io as nio
from npge_amd.model import blockset_hash

GOLD = os.path.join(os.path.dirname(__file__), "golden")

SCRIPTS = {
    # Read; RemoveAlignment; MetaAligner with the similar aligner; RawWrite
    "align": "run_main 'Read'\nrun 'RemoveAlignment'\n"
             "run('MetaAligner', '--aligner-type=similar')\nrun_main 'RawWrite'\n",
    # anchors into `other` (repeated: the reference's Bloom parameters differ
    # run to run), their overlap-free union into `target`, Write
    "anchor_finder": "run_main('Read', 'target=other')\n"
                     "for i = 1, 15 do\n    run('AnchorFinder', '--anchor-size:=20 target=other') -- anchors\nend\n"
                     "run('OverlaplessUnion', 'target=target other=other')\n"
                     "run_main('Write', '--skip-rest:=1')\n",
    "filter": "run_main('Read')\nrun('Filter', '--find-subblocks=1 --min-identity=1')\nrun_main('RawWrite')\n",
    "stem": "run_main('Read')\nrun('RemoveNonStem', '--exact=0')\nrun_main('RawWrite')\n",
    # Read; CutGaps permissive / strict; RawWrite
    "cut_gaps": "run_main('Read')\nrun('CutGaps', '--cut-strict=0')\nrun_main('RawWrite')\n",
    "cut_gaps_strict": "run_main('Read')\nrun('CutGaps', '--cut-strict=1')\nrun_main('RawWrite')\n",
    "stem-exact": "bs1 = BlockSet.new()\nRead {target=bs1}\nRemoveNonStem {target=bs1, exact=true}\n"
                  "RawWrite {target=bs1}\n",
}

CASES = [(s, c) for s in SCRIPTS for c in sorted(os.listdir(os.path.join(GOLD, s)))
         if os.path.exists(os.path.join(GOLD, s, c, "out.fasta"))]


@pytest.mark.gpu
@pytest.mark.parametrize("script,case", CASES)
def test_script_fixture(script, case):
    from npge_amd.script import output_hash, run_script
    d = os.path.join(GOLD, script, case)
    out = run_script(SCRIPTS[script], open(os.path.join(d, "in.fasta")).read())
    exp = nio.read_blockset(open(os.path.join(d, "out.fasta")).read())
    want = blockset_hash(exp.blocks)
    assert output_hash(out) == want
    if script.startswith("cut_gaps"):  # the rows too
        assert sorted((f.id(), f.row) for b in out.blocks for f in b.fragments) == \
            sorted((f.id(), f.row) for b in exp.blocks for f in b.fragments)
    if want == 0:  # (meta_test only warns on an empty expected set: compare the fragments too)
        assert sorted(f.id() for b in out.blocks for f in b.fragments) == \
            sorted(f.id() for b in exp.blocks for f in b.fragments)


def test_script_grammar_on_cpu():
    """Parsing and the bookkeeping processors (no GPU): comments outside
    strings, string-call sugar, the for loop, table calls, set mapping."""
    from npge_amd.script import Script
    text = open(os.path.join(GOLD, "align", "1", "in.fasta")).read()
    s = Script(text)
    out = s.run("-- a comment\nx = BlockSet.new()\nRead {target=x}\nfor i = 1, 2 do\n"
                "  run('RemoveAlignment', 'target=x') -- '--' inside a comment\nend\n"
                "run_main('RawWrite', 'target=x --skip-rest:=1')\n")
    assert out.blocks and out.blocks[0].fragments[0].seq is s.sets["x"].blocks[0].fragments[0].seq
    assert all(f.row is None for b in out.blocks for f in b.fragments)
    assert s.sets["target"].blocks == []
    # Read / Write see the program arguments only under run_main (lua_lib.lua:100-133);
    # the written set is a snapshot
    s2 = Script(text)
    assert s2.run("run('Read')\nrun('RawWrite')\n") is None
    assert s2.sets["target"].blocks == []
    s3 = Script(text)
    out = s3.run("run_main('Read')\nrun_main('RawWrite')\nrun('RemoveAlignment')\n")
    assert all(f.row is not None for b in out.blocks for f in b.fragments)
