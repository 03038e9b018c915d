"""FASTA / .bs helpers (the part of src/algo/Read.cpp, RawWrite.cpp and
FastaReader the hot path's fixtures need; SURVEY.md §8 f rank 3).

A ``.bs`` file is FASTA whose headers are fragment ids ``seq_begin_last`` with
``block=NAME`` in the description; sequences are headers without a fragment-id
shape (Fragment.cpp:329-341, Sequence.cpp:116-149).
"""
import re

from .model import Block, BlockSet, Fragment, Sequence

_IUPAC_N = set("RYMKWSBVHD")


def to_atgcn(s: str) -> str:
    """Sequence::to_atgcn Sequence.cpp:151-179."""
    out = []
    for c in s.upper():
        if c in "ATGCN":
            out.append(c)
        elif c in _IUPAC_N:
            out.append("N")
    return "".join(out)


def read_fasta(text):
    """Yield (name, description, raw_sequence_text) records."""
    name = None
    desc = ""
    chunks = []
    for line in text.splitlines():
        if line.startswith(">"):
            if name is not None:
                yield name, desc, "".join(chunks)
            head = line[1:].strip()
            parts = head.split(None, 1)
            name = parts[0] if parts else ""
            desc = parts[1] if len(parts) > 1 else ""
            chunks = []
        else:
            chunks.append(line.strip())
    if name is not None:
        yield name, desc, "".join(chunks)


_FRAG_RE = re.compile(r"^(.+)_(-?\d+)_(-?\d+)$")


def parse_fragment_id(fid):
    """Inverse of Fragment::id (Fragment.cpp:173-183): returns
    (seq_name, min_pos, max_pos, ori) or None."""
    m = _FRAG_RE.match(fid)
    if not m:
        return None
    name, a, b = m.group(1), int(m.group(2)), int(m.group(3))
    if b == -1:
        return name, a, a, -1
    if a <= b:
        return name, a, b, 1
    return name, b, a, -1


def read_blockset(text):
    """Read sequences and blocks (with rows when the record is gapped) from a
    .bs/FASTA text.  Sequences: records without a block= description."""
    bs = BlockSet()
    seq_by_name = {}
    frag_recs = []
    for name, desc, raw in read_fasta(text):
        m = re.search(r"block=(\S+)", desc)
        if m:
            frag_recs.append((name, m.group(1), raw, "norow" in desc))
        else:
            s = Sequence(name, to_atgcn(raw), desc)
            bs.seqs.append(s)
            seq_by_name[name] = s
    blocks = {}
    for fid, bname, raw, norow in frag_recs:
        p = parse_fragment_id(fid)
        if p is None:
            continue
        sname, mn, mx, ori = p
        seq = seq_by_name.get(sname)
        if seq is None:
            # fragment-only file (e.g. expected outputs): synthesise a name-only sequence
            seq = Sequence(sname, "")
            seq_by_name[sname] = seq
        row = None if norow else raw.upper()
        f = Fragment(seq, mn, mx, ori, row)
        blocks.setdefault(bname, Block(name=bname)).fragments.append(f)
    bs.blocks = list(blocks.values())
    return bs


def write_blockset(bs, with_rows=True):
    """RawWrite-like output: sequences, then block fragments."""
    out = []
    for s in bs.seqs:
        out.append(">%s %s" % (s.name, s.description) if s.description else ">%s" % s.name)
        out.append(s.data)
    for b in bs.blocks:
        for f in b.fragments:
            if with_rows and f.row is not None:
                out.append(">%s block=%s" % (f.id(), b.name))
                out.append(f.row)
            else:
                out.append(">%s block=%s norow" % (f.id(), b.name))
                out.append(f.str())
    return "\n".join(out) + "\n"
