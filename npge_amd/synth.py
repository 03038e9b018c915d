"""Seeded synthetic genome sets (BASELINE.md "Inputs", SURVEY.md §8 d).

The Brucella FASTA files are not available offline (examples/Brucella/*.tsv
only list EMBL accessions), so every config runs on a Brucella-like proxy:
a random root genome, and per genome substitutions at rate d with ~10% of the
events indels of 1-10 nt, plus 0-3 N runs of 50-500 nt per chromosome.  Genome
lengths are made distinct (+17*i nt) to avoid the reference's size-tie
ambiguity (SeqI.hpp:54).  Names are ``Gxx&chrY&c`` so Sequence::genome()
parses them (Sequence.cpp:193-202).
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

BASE_SEED = 20261015


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
    names, seqs = [], []
    lengths = set()
    for g in range(n_genomes):
        for c, root in enumerate(roots):
            codes = _mutate(rng, root, d) if g > 0 else root.copy()
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
