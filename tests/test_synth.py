"""The synthetic genome sets (npge_amd/synth.py): seeded and reproducible, the
plain configs' byte content pinned (the full-size fixtures depend on it), and
the repeat-rich configs carry element families in many copies per genome."""
import hashlib

from npge_amd import synth


def _sha(seqs):
    return hashlib.sha1("".join(seqs).encode()).hexdigest()[:12]


def test_plain_configs_pinned():
    assert _sha(synth.genome_set("tiny")[1]) == "8f2507960dcd"
    assert _sha(synth.genome_set("small")[1]) == "d2e6669247fb"


def test_repeat_configs():
    names, seqs = synth.genome_set("rsmall")
    assert names == synth.genome_set("rsmall")[0] and seqs == synth.genome_set("rsmall")[1]
    assert len(seqs) == 10
    # 20-mers that occur many times across the set: the element copies
    from collections import Counter
    c = Counter()
    for s in seqs[::2]:  # chromosome 1 of each genome
        for i in range(0, len(s) - 20, 7):
            c[s[i:i + 20]] += 1
    top = c.most_common(1)[0][1]
    assert top >= 5 * 3  # several copies per genome of one element family
