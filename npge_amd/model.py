"""Host-side block-set model: the minimum of NPG-explorer's model layer the hot
path produces and consumes.

* ``Fragment``  -- (sequence, min_pos, max_pos, ori) + optional gapped row
  (src/model/Fragment.hpp; id format Fragment.cpp:173-183).
* ``Block``     -- ordered list of fragments (Block.hpp:41).
* ``BlockSet``  -- sequences + blocks (BlockSet.hpp:30).
* ``block_hash`` / ``blockset_hash`` -- the order-independent, coordinate-only
  comparison the reference's script tests use (block_hash.cpp:29-55,125-130).
"""
from dataclasses import dataclass, field
from typing import List, Optional

MASK64 = (1 << 64) - 1


@dataclass
class Sequence:
    name: str
    data: str            # after to_atgcn (Sequence.cpp:151-179)
    description: str = ""
    # the block whose consensus this sequence holds (Sequence::set_block,
    # Sequence.cpp:301-335; set by ConSeq, read by DeConSeq)
    block: Optional["Block"] = field(default=None, repr=False, compare=False)

    def size(self):
        return len(self.data)

    def genome(self):
        """Sequence.cpp:193-202."""
        parts = self.name.split("&")
        if len(parts) == 3 and parts[2] in ("c", "l"):
            return parts[0]
        return ""


_COMPL = str.maketrans("ATGCatgc", "TACGtacg")


def complement(s: str) -> str:
    """Reverse complement, other chars (N, '-') unchanged (complement.hpp:19-32)."""
    return s.translate(_COMPL)[::-1]


@dataclass
class Fragment:
    seq: Sequence
    min_pos: int
    max_pos: int
    ori: int = 1
    row: Optional[str] = None   # gapped row ('-' = gap), None = no alignment

    def length(self):
        return self.max_pos - self.min_pos + 1

    def begin_pos(self):
        return self.min_pos if self.ori == 1 else self.max_pos

    def last_pos(self):
        return self.max_pos if self.ori == 1 else self.min_pos

    def id(self):
        """Fragment::id Fragment.cpp:173-183."""
        a, b = self.begin_pos(), self.last_pos()
        if a == b and self.ori == -1:
            b = -1
        return "%s_%d_%d" % (self.seq.name, a, b)

    def inverse_id(self):
        f = Fragment(self.seq, self.min_pos, self.max_pos, -self.ori)
        return f.id()

    def str(self):
        s = self.seq.data[self.min_pos:self.max_pos + 1]
        return s if self.ori == 1 else complement(s)

    def key(self):
        return (self.seq.name, self.min_pos, self.max_pos, self.ori)


@dataclass
class Block:
    fragments: List[Fragment] = field(default_factory=list)
    name: str = ""

    def size(self):
        return len(self.fragments)

    def alignment_length(self):
        if not self.fragments:
            return 0
        f = self.fragments[0]
        return len(f.row) if f.row is not None else f.length()


@dataclass
class BlockSet:
    seqs: List[Sequence] = field(default_factory=list)
    blocks: List[Block] = field(default_factory=list)


def block_hash(block: Block) -> int:
    """block_hash block_hash.cpp:29-55 (uint64 arithmetic, little-endian words)."""
    ids_dir = sorted(f.id() for f in block.fragments)
    ids_inv = sorted(f.inverse_id() for f in block.fragments)
    ids = ids_dir if ids_dir < ids_inv else ids_inv
    joint = " ".join(ids).encode()
    loop = 16
    new_size = (len(joint) + loop - 1) // loop * loop
    joint = joint + b" " * (new_size - len(joint))
    a = 1
    for i in range(len(joint) // loop):
        v0 = int.from_bytes(joint[16 * i:16 * i + 8], "little")
        v1 = int.from_bytes(joint[16 * i + 8:16 * i + 16], "little")
        a = (a * v0) & MASK64
        a ^= v1
    return a


def blockset_hash(blocks) -> int:
    """blockset_hash block_hash.cpp:112-130: XOR over blocks with >= 2 fragments."""
    h = 0
    for b in blocks:
        if b.size() > 1:
            h ^= block_hash(b)
    return h


def normalized_blocks(blocks):
    """Order-independent canonical form (set of sorted id tuples, inverse-
    normalised like block_hash) for readable test diffs."""
    out = set()
    for b in blocks:
        if b.size() <= 1:
            continue
        d = tuple(sorted(f.id() for f in b.fragments))
        i = tuple(sorted(f.inverse_id() for f in b.fragments))
        out.add(min(d, i))
    return out
