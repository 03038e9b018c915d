"""Shared test helpers."""
from npge_amd.model import Block, Fragment


def af_blocks_from_result(r, seqs):
    """SoA anchor result -> list of Block (fragments in result order)."""
    blocks = []
    bs = r["block_start"]
    for b in range(len(bs) - 1):
        frs = [Fragment(seqs[int(r["seq"][i])], int(r["min_pos"][i]), int(r["max_pos"][i]),
                        int(r["ori"][i])) for i in range(bs[b], bs[b + 1])]
        blocks.append(Block(frs))
    return blocks
