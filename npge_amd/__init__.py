"""npge_amd -- MI355X-native anchor finding and greedy multiple alignment for
NPG-explorer's block-construction hot path."""
