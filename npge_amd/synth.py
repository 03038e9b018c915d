"""Seeded synthetic genome sets (BASELINE.md "Inputs", SURVEY.md §8 d).

The Brucella FASTA files are not available offline (examples/Brucella/*.tsv
only list EMBL accessions), so every config runs on a Brucella-like proxy:
a random root genome, and per genome substitutions at rate d with ~10% of the
events indels of 1-10 nt, plus 0-3 N runs of 50-500 nt per chromosome.  Genome
lengths are made distinct (+17*i nt) to avoid the reference's size-tie
ambiguity (SeqI.hpp:54).  Names are ``Gxx&chrY&c`` so Sequence::genome()
parses them (Sequence.cpp:193-202).

Repeat-rich, rearranged sets (REPEATS; VERDICT r03 #7, the reference's own
randomized test plants repeats, src/test/test_repeats.sh.in:1-30, and real
Brucella carries IS-element families): IS-like element families (a random
consensus of `elem_len` nt per family, every copy 1-3 % away from it) are
planted in the root -- ancestral copies every genome inherits and then
mutates -- plus genome-specific copies of their own; each genome then gets
0..max_inv inversions (reverse complement of a 5-50 kb segment).  Anchor
groups then hold copies x genomes fragments and the aligner sees alignment
problems of more than 64 rows (the wide path).  The repeat draws use their own
random stream, so the plain configs are unchanged.
"""
import numpy as np

LETTERS = np.frombuffer(b"ATGC", dtype=np.uint8)

CONFIGS = {
    # name: (n_genomes, chromosome lengths, divergence)
    "C1": (3, (2_120_000, 1_180_000), 0.008),
    "C2": (3, (2_120_000, 1_180_000), 0.008),
    "C3": (17, (2_120_000, 1_180_000), 0.008),
    "C4": (32, (5_000_000,), 0.02),
    "C5": (8, (50_000_000,), 0.01),
    "tiny": (3, (20_000, 11_000), 0.008),
    "small": (5, (200_000, 110_000), 0.008),
}

# name: (families, element length, ancestral copies per family, extra copies per
# genome and family (0..max), inversions per genome (0..max), inversion length range)
REPEATS = {
    "R3": (4, 1300, 24, 16, 3, (5_000, 50_000)),      # C3-shaped: 17 genomes, 24-40 copies of 4 families
    "rtiny": (2, 300, 3, 2, 1, (1_000, 3_000)),
    "rsmall": (2, 600, 10, 48, 1, (2_000, 8_000)),    # 5 genomes, 10 ancestral + 0-48 own copies: > 64-row problems
}
CONFIGS.update({
    "R3": (17, (2_120_000, 1_180_000), 0.008),
    "rtiny": (3, (20_000, 11_000), 0.008),
    "rsmall": (5, (200_000, 110_000), 0.008),
})

BASE_SEED = 20261015
_COMP = np.array([1, 0, 3, 2], dtype=np.uint8)  # codes A0 T1 G2 C3 -> complement


def _element_copy(rng, cons):
    """One copy of an element family: 1-3 % substitutions from the consensus."""
    c = cons.copy()
    d = float(rng.uniform(0.01, 0.03))
    hit = np.flatnonzero(rng.random(len(c)) < d)
    c[hit] = (c[hit] + rng.integers(1, 4, len(hit))) % 4
    return c if rng.random() < 0.5 else _COMP[c[::-1]]  # either strand


def _plant(rng, codes, copies):
    """Inserts the element copies at random positions of codes."""
    if not copies:
        return codes
    pos = np.sort(rng.integers(0, len(codes), len(copies)))
    pieces, prev = [], 0
    for p, c in zip(pos.tolist(), copies):
        pieces.append(codes[prev:p])
        pieces.append(c)
        prev = p
    pieces.append(codes[prev:])
    return np.concatenate(pieces)


def _invert(rng, codes, max_inv, inv_range):
    for _ in range(int(rng.integers(0, max_inv + 1))):
        n = int(rng.integers(inv_range[0], inv_range[1] + 1))
        if n >= len(codes):
            continue
        a = int(rng.integers(0, len(codes) - n))
        codes = codes.copy()
        codes[a:a + n] = _COMP[codes[a:a + n][::-1]]
    return codes


def _mutate(rng, root, d):
    L = len(root)
    ev = np.flatnonzero(rng.random(L) < d)
    is_indel = rng.random(len(ev)) < 0.1
    sub = ev[~is_indel]
    out = root.copy()
    out[sub] = (out[sub] + rng.integers(1, 4, len(sub))) % 4
    indels = ev[is_indel]
    if len(indels) == 0:
        return out
    pieces = []
    prev = 0
    for p in indels:
        if p < prev:
            continue
        n = int(rng.integers(1, 11))
        pieces.append(out[prev:p])
        if rng.random() < 0.5:
            pieces.append(rng.integers(0, 4, n).astype(np.uint8))  # insertion
            prev = p
        else:
            prev = min(L, p + n)                                   # deletion
    pieces.append(out[prev:])
    return np.concatenate(pieces)


def genome_set(config="C2", seed=None):
    """Returns (names, sequences as str)."""
    n_genomes, chrom_lens, d = CONFIGS[config]
    seed = BASE_SEED + sum(map(ord, config)) if seed is None else seed
    rng = np.random.default_rng(seed)
    roots = [rng.integers(0, 4, L).astype(np.uint8) for L in chrom_lens]
    rep = REPEATS.get(config)
    if rep is not None:  # repeat families and inversions (their own random stream)
        fam, elen, anc, extra_max, max_inv, inv_range = rep
        rr = np.random.default_rng(seed ^ 0x5EED)
        cons = [rr.integers(0, 4, elen).astype(np.uint8) for _ in range(fam)]
        total = sum(chrom_lens)
        roots = [_plant(rr, root, [_element_copy(rr, cons[f]) for f in range(fam)
                                   for _ in range(int(round(anc * len(root) / total)))]) for root in roots]
    names, seqs = [], []
    lengths = set()
    for g in range(n_genomes):
        for c, root in enumerate(roots):
            codes = _mutate(rng, root, d) if g > 0 else root.copy()
            if rep is not None and g > 0:  # genome-specific copies, then inversions
                share = len(root) / sum(len(r) for r in roots)
                codes = _plant(rr, codes, [_element_copy(rr, cons[f]) for f in range(fam)
                                           for _ in range(int(rr.integers(0, int(extra_max * share) + 1)))])
                codes = _invert(rr, codes, max_inv, inv_range)
            extra = rng.integers(0, 4, 17 * g + c).astype(np.uint8)
            codes = np.concatenate([codes, extra])
            while len(codes) in lengths:
                codes = np.concatenate([codes, rng.integers(0, 4, 1).astype(np.uint8)])
            lengths.add(len(codes))
            text = LETTERS[codes]
            for _ in range(int(rng.integers(0, 4))):
                run = int(rng.integers(50, 501))
                start = int(rng.integers(0, max(1, len(text) - run)))
                text[start:start + run] = ord("N")
            names.append("G%02d&chr%d&c" % (g + 1, c + 1))
            seqs.append(text.tobytes().decode())
    return names, seqs


def total_bp(seqs):
    return sum(len(s) for s in seqs)
