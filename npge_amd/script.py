"""Fixed-form ``script.npge`` runner over the Processor mirror.

NPG-explorer's test harness (src/test/meta_test.cxx:53-102) runs every
``test-script/<case>/script.npge`` with ``--in-blocks <dir>/in.fasta
--out-file <tmp>`` and compares ``hash_block_sets`` of the output with that
of ``out.fasta``.  The scripts are Lua; Lua is not available here, so this
module interprets the fixed-form subset those scripts use:

* ``run_main('Name', 'opts')`` / ``run_main 'Name'`` -- a processor that
  also sees the program arguments (lua_lib.lua:100-126): ``Read`` reads
  ``--in-blocks``, ``Write`` / ``RawWrite`` write ``--out-file``;
* ``run('Name', 'opts')`` / ``run 'Name'`` (lua_lib.lua:128-133);
* ``for i = a, b do ... end`` (constant bounds);
* ``x = BlockSet.new()`` and the table-call form ``Name {target=x, opt=v}``;
* ``--`` comments.

Option strings follow Processor::set_options (``--opt=v``, ``--opt:=v``,
``target=name``); block-set names resolve in one namespace per script, with
``target`` and ``other`` as the main program's two sets.  The compute-heavy
processors run on the HIP library (BlockSetEngine, AnchorFinder); the
registered ones here are the I/O and bookkeeping around them.
"""
import re

from . import anchor_finder, conseq  # noqa: F401  (register AnchorFinder, ConSeq, DeConSeq)
from . import io as nio
from .model import Block, BlockSet, Fragment, Sequence, blockset_hash
from .processor import Decimal, OptionError, Processor, new_p, register


# ------------------------------------------------------------------ processors
class _EngineProcessor(Processor):
    """A processor whose block work is one npgx_blockset_apply call."""

    engine_name = None

    def engine_kwargs(self):
        return {}

    def engine_processor(self):
        return self.engine_name

    def run_impl(self):
        from . import _capi
        from .blockset import BlockSetEngine
        bs = self.block_set()
        if not bs.blocks:
            return
        known = {id(s) for s in bs.seqs}
        for b in bs.blocks:  # sequences named only by fragments (fragment-only files)
            for f in b.fragments:
                if id(f.seq) not in known:
                    known.add(id(f.seq))
                    bs.seqs.append(f.seq)
        _complete_sequences(bs)
        index = {id(s): i for i, s in enumerate(bs.seqs)}
        blocks = [[(index[id(f.seq)], f.min_pos, f.max_pos, f.ori, f.row) for f in b.fragments]
                  for b in bs.blocks]
        ss = _capi.SeqSet([s.data for s in bs.seqs], [s.name for s in bs.seqs])
        eng = BlockSetEngine(ss, **self.engine_kwargs())
        eng.set_blocks(blocks).apply(self.engine_processor())
        bs.blocks = [Block([Fragment(bs.seqs[q], mn, mx, ori, row) for q, mn, mx, ori, row in blk])
                     for blk in eng.blocks()]


@register
class MetaAligner(_EngineProcessor):
    """MetaAligner (MetaAligner.cpp): every unaligned block aligned."""
    name = "MetaAligner"
    engine_name = "MetaAligner"

    def __init__(self):
        super().__init__()
        self.add_gopt("aligner-type", "aligner (the engine's: similar)", "ALIGNER")
        self.add_opt_rule("aligner-type = similar", lambda p: p.opt_value("aligner-type") == "similar")


@register
class Align(MetaAligner):
    """Align (Align.cpp:36-52): MetaAligner, SelfOverlapsResolver,
    MetaAligner, then {MoveGaps, CutGaps, Filter} until the block set repeats."""
    name = "Align"
    engine_name = "Align"


@register
class LiteAlign(MetaAligner):
    """LiteAlign (Align.cpp:17-30): MetaAligner, then {MoveGaps, CutGaps}."""
    name = "LiteAlign"
    engine_name = "LiteAlign"


@register
class MoveGaps(_EngineProcessor):
    """MoveGaps (MoveGaps.cpp:21-103): terminal letters moved inside."""
    name = "MoveGaps"

    def __init__(self):
        super().__init__()
        self.add_gopt("max-tail", "Max length of tail", "MAX_TAIL")
        self.add_gopt("max-tail-to-gap", "Max tail length to gap length ratio", "MAX_TAIL_TO_GAP", Decimal)

    def engine_processor(self):
        d = self.opt_value("max-tail-to-gap").impl
        return "MoveGaps --max-tail=%d --max-tail-to-gap=%d.%04d" % (self.opt_value("max-tail"), d // 10000,
                                                                     d % 10000)


@register
class CutGaps(_EngineProcessor):
    """CutGaps (CutGaps.cpp:20-159): terminal gap columns cut."""
    name = "CutGaps"

    def __init__(self):
        super().__init__()
        self.add_opt("cut-strict", "cut more gaps", False)

    def engine_processor(self):
        return "CutGaps --cut-strict=%d" % int(bool(self.opt_value("cut-strict")))


@register
class SelfOverlapsResolver(_EngineProcessor):
    """SelfOverlapsResolver (SelfOverlapsResolver.cpp:19-22, hit.cpp:68-91)."""
    name = "SelfOverlapsResolver"
    engine_name = "SelfOverlapsResolver"


@register
class Filter(_EngineProcessor):
    """Filter (Filter.cpp:129-277)."""
    name = "Filter"
    engine_name = "Filter"

    def __init__(self):
        super().__init__()
        self.add_gopt("min-identity", "minimum identity of a good column frame", "MIN_IDENTITY", Decimal)
        self.add_opt("find-subblocks", "find good sub-blocks", True)

    def engine_kwargs(self):
        return {"min_identity_x1e4": self.opt_value("min-identity").impl,
                "find_subblocks": int(bool(self.opt_value("find-subblocks")))}


@register
class RemoveNonStem(_EngineProcessor):
    """RemoveNonStem (RemoveNonStem.cpp:29-45)."""
    name = "RemoveNonStem"

    def __init__(self):
        super().__init__()
        self.add_opt("exact", "exactly one fragment of every genome", False)

    def engine_processor(self):
        return "RemoveNonStem --exact" if self.opt_value("exact") else "RemoveNonStem"


@register
class OverlaplessUnion(_EngineProcessor):
    """OverlaplessUnion (OverlaplessUnion.cpp:54-80): clones of other's blocks
    that overlap nothing in target, largest first.  The engine admits the
    blocks of one set against each other, so target must start empty here."""
    name = "OverlaplessUnion"
    engine_name = "OverlaplessUnion"

    def run_impl(self):
        t, o = self.block_set(), self.other()
        if t is o:
            return
        if t.blocks:
            raise OptionError("OverlaplessUnion: the fixed-form runner needs an empty target")
        for s in o.seqs:
            if all(s is not x for x in t.seqs):
                t.seqs.append(s)
        t.blocks = [Block([Fragment(f.seq, f.min_pos, f.max_pos, f.ori, f.row) for f in b.fragments],
                          name=b.name) for b in o.blocks]
        super().run_impl()


@register
class ExtendLoop(_EngineProcessor):
    """The ExtendLoop pipe (lua_lib.lua:677-688) to its fixpoint: MoveUnchanged,
    ExtendAndAlign, AddingLoopBySize, until the block set repeats."""
    name = "ExtendLoop"
    engine_name = "ExtendLoop"


@register
class AddingLoopBySize(_EngineProcessor):
    """AddingLoopBySize (TrySmth.cpp:157-178): Align other's blocks and move
    the overlapless ones (cut where they overlap) into target, until other is
    empty.  The engine starts from an empty target, so target must be empty
    here; other ends empty."""
    name = "AddingLoopBySize"
    engine_name = "AddingLoopBySize"

    def run_impl(self):
        t, o = self.block_set(), self.other()
        if t is o:
            super().run_impl()
            return
        if t.blocks:
            raise OptionError("AddingLoopBySize: the fixed-form runner needs an empty target")
        for sq in o.seqs:
            if all(sq is not x for x in t.seqs):
                t.seqs.append(sq)
        t.blocks, o.blocks = o.blocks, []
        super().run_impl()


@register
class RemoveAlignment(Processor):
    """RemoveAlignment: every fragment loses its row."""
    name = "RemoveAlignment"

    def run_impl(self):
        for b in self.block_set().blocks:
            for f in b.fragments:
                f.row = None


@register
class Read(Processor):
    """Read (Read.cpp:36-64): the program's --in-blocks text when run as the
    main program (run_main, lua_lib.lua:100-126); no input otherwise."""
    name = "Read"
    in_text = ""

    def run_impl(self):
        if not self.in_text:
            return
        src = nio.read_blockset(self.in_text)
        bs = self.block_set()
        bs.seqs.extend(src.seqs)
        bs.blocks.extend(src.blocks)


@register
class RawWrite(Processor):
    """RawWrite (RawWrite.cpp:40-59) to the program's --out-file when run as
    the main program: the script keeps a snapshot of the set as written (its
    text: npge_amd.io.write_blockset); later statements do not change it."""
    name = "RawWrite"
    written = None

    def __init__(self):
        super().__init__()
        self.add_opt("skip-rest", "write only blocks", False)

    def run_impl(self):
        bs = self.block_set()
        snap = BlockSet()
        snap.seqs = list(bs.seqs)
        snap.blocks = [Block([Fragment(f.seq, f.min_pos, f.max_pos, f.ori, f.row) for f in b.fragments],
                             name=b.name) for b in bs.blocks]
        self.written = snap


@register
class Write(RawWrite):
    name = "Write"


_COMP = {"A": "T", "T": "A", "G": "C", "C": "G", "N": "N"}


def _complete_sequences(bs):
    """Fragment-only inputs (the expected-output style fixtures) name their
    sequences without text: give each one text long enough for its fragments,
    the rows' letters where rows cover it and 'A' elsewhere."""
    need = {}  # id(sequence) -> [sequence, length needed]
    for b in bs.blocks:
        for f in b.fragments:
            if not f.seq.data:
                entry = need.setdefault(id(f.seq), [f.seq, 0])
                entry[1] = max(entry[1], f.max_pos + 1)
    for seq, n in need.values():
        text = ["A"] * n
        for b in bs.blocks:
            for f in b.fragments:
                if f.seq is not seq or f.row is None:
                    continue
                letters = [c for c in f.row if c != "-"]
                if f.ori == -1:
                    letters = [_COMP.get(c, "N") for c in reversed(letters)]
                for i, c in enumerate(letters[:f.max_pos - f.min_pos + 1]):
                    text[f.min_pos + i] = c
        seq.data = "".join(text)


# ------------------------------------------------------------------ interpreter
_STR = r"""(?:'((?:[^'\\]|\\.)*)'|"((?:[^"\\]|\\.)*)")"""


def _strings(s):
    """The string literals of s, in order."""
    return [m.group(1) if m.group(1) is not None else m.group(2) for m in re.finditer(_STR, s)]


def _strip_comment(line):
    """line without its Lua comment (-- outside string literals)."""
    q = None
    for i, c in enumerate(line):
        if q:
            if c == q:
                q = None
        elif c in "'\"":
            q = c
        elif line.startswith("--", i):
            return line[:i]
    return line


class Script:
    """One script run: block-set namespace, the program arguments, the output."""

    def __init__(self, in_text):
        self.sets = {"target": BlockSet(), "other": BlockSet()}
        self.in_text = in_text
        self.out = None

    def _proc(self, name, opts, main):
        p = new_p(name)
        if isinstance(p, Read) and main:  # only run_main passes the program arguments
            p.in_text = self.in_text
        if isinstance(opts, dict):
            for k, v in opts.items():
                if k in ("target", "other"):
                    p.set_bs(k, self.sets.setdefault(v, BlockSet()))
                else:
                    p.set_opt_value(k.replace("_", "-"), v)
            for k in ("target", "other"):
                if k not in opts:
                    p.set_bs(k, self.sets[k])
        else:
            p.set_bs("target", self.sets["target"])
            p.set_bs("other", self.sets["other"])
            p.set_options(opts, self.sets)
        p.run()
        if isinstance(p, RawWrite) and main:
            self.out = p.written
        return p

    def run(self, text):
        stmts = [t for t in (_strip_comment(ln).strip() for ln in text.splitlines()) if t]
        self._block(stmts, 0, len(stmts))
        return self.out

    def _block(self, stmts, i, end):
        while i < end:
            st = stmts[i]
            m = re.match(r"for\s+\w+\s*=\s*(-?\d+)\s*,\s*(-?\d+)\s+do$", st)
            if m:
                depth, j = 1, i + 1
                while j < end and depth:
                    if re.match(r"for\s.*\sdo$", stmts[j]):
                        depth += 1
                    elif stmts[j] == "end":
                        depth -= 1
                    j += 1
                for _ in range(int(m.group(1)), int(m.group(2)) + 1):
                    self._block(stmts, i + 1, j - 1)
                i = j
                continue
            self._statement(st)
            i += 1

    def _statement(self, st):
        m = re.match(r"(run_main|run)\s*(\(.*\)|" + _STR + r")$", st)
        if m:
            args = _strings(m.group(2))
            self._proc(args[0], args[1] if len(args) > 1 else "", m.group(1) == "run_main")
            return
        m = re.match(r"(\w+)\s*=\s*BlockSet\.new\(\)$", st)
        if m:
            self.sets[m.group(1)] = BlockSet()
            return
        m = re.match(r"(\w+)\s*\{(.*)\}$", st)
        if m:
            opts = {}
            for kv in filter(None, (x.strip() for x in m.group(2).split(","))):
                k, v = (x.strip() for x in kv.split("=", 1))
                sv = _strings(v)
                opts[k] = sv[0] if sv else {"true": True, "false": False}.get(v, v)
            self._proc(m.group(1), opts, True)
            return
        raise OptionError("script.npge: unsupported statement: " + st)


def run_script(script_text, in_text):
    """Runs a fixed-form script on the --in-blocks text; returns the BlockSet
    written by its Write/RawWrite (None if it wrote nothing)."""
    return Script(in_text).run(script_text)


def output_hash(bs):
    """hash_block_sets of the written set (blockset_hash of its blocks)."""
    return blockset_hash(bs.blocks) if bs is not None else 0


__all__ = ["run_script", "output_hash", "Script", "Sequence"]
