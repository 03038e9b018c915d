"""ConSeq / DeConSeq processors (src/algo/ConSeq.cpp:20-65,
src/algo/DeConSeq.cpp:20-107) on the host model (npge_amd.model), computed by
the HIP engine: npgx_blockset_conseq (consensus of aligned blocks on the GPU)
and npgx_blockset_deconseq.  Used by AnchorLoopFast (lua_lib.lua:741-756) to
run AnchorFinder on block consensuses and map the anchors back."""
from .blockset import BlockSetEngine
from .model import Block, Fragment, Sequence
from .processor import Processor, register
from . import _capi


def _engine(seqs, blocks):
    """Engine over `seqs` (model Sequences) holding `blocks` (model Blocks)."""
    idx = {id(s): i for i, s in enumerate(seqs)}
    ss = _capi.SeqSet([s.data for s in seqs], [s.name for s in seqs])
    eng = BlockSetEngine(ss)
    eng.set_blocks([[(idx[id(f.seq)], f.min_pos, f.max_pos, f.ori, f.row) for f in b.fragments]
                    for b in blocks])
    return eng


@register
class ConSeq(Processor):
    """ConSeq (ConSeq.cpp:20-57): every block of `other` becomes a sequence of
    `target` -- its consensus (two or more fragments) or the fragment itself --
    bound to the block (Sequence::set_block) and named after it."""
    name = "ConSeq"

    def run_impl(self):
        other, target = self.other(), self.block_set()
        blocks = [b for b in other.blocks if b.fragments]
        if not blocks:
            return
        texts = _engine(other.seqs, blocks).conseq()
        for b, t in zip(blocks, texts):
            target.seqs.append(Sequence(name=b.name, data=t, block=b))


@register
class DeConSeq(Processor):
    """DeConSeq (DeConSeq.cpp:20-107): every block of `other` (over ConSeq's
    consensus sequences) becomes a block of `target` over the original
    sequences (Block::slice of the consensus' block, rows composed)."""
    name = "DeConSeq"

    def run_impl(self):
        other, target = self.other(), self.block_set()
        if not other.blocks:
            return
        for s in other.seqs:
            if s.block is None:
                raise _capi.NpgxError(-5, "Sequence " + s.name + " is not bound to a block")
        src_blocks = [s.block for s in other.seqs]
        seqs = list(target.seqs)
        known = {id(s) for s in seqs}
        for b in src_blocks:
            for f in b.fragments:
                if id(f.seq) not in known:
                    known.add(id(f.seq))
                    seqs.append(f.seq)
        src = _engine(seqs, src_blocks)
        cons = _engine(other.seqs, other.blocks)
        out = _engine(seqs, [])
        out.deconseq(cons, source=src)
        new = out.blocks()
        # one new block per consensus block, in order (empty ones included,
        # DeConSeq.cpp:94-99): each keeps its consensus block's name
        if len(new) != len(other.blocks):
            raise _capi.NpgxError(-5, "DeConSeq: %d blocks for %d consensus blocks" % (len(new), len(other.blocks)))
        for blk, name in zip(new, [b.name for b in other.blocks]):
            target.blocks.append(Block([Fragment(seqs[q], mn, mx, ori, row) for q, mn, mx, ori, row in blk],
                                       name=name))
