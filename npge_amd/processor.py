"""Processor plugin surface for the hot path, mirroring NPG-explorer's.

The reference plugin interface is the C++ class ``Processor``
(src/algo/Processor.hpp:42-510): options registered with add_opt/add_gopt and
checked with option rules, named block sets ("target", "other"), ``run()``
calling ``run_impl()``; the Lua layer adds ``new_p(name)``, ``run(name, opts)``
and option strings such as ``'--anchor-size:=20 target=other'``
(src/algo/lua_lib.lua:59-133, grammar Processor.cpp:260-322).  Lua itself is not
available here, so the same call shapes are offered from Python; the compute
behind them is the HIP library (npge_amd._capi), never a CPU fallback.
"""
import shlex

from .model import BlockSet

# Compile-time global defaults (CMakeLists.txt:31-60 -> opts_lib.cpp.in)
GLOBAL_OPTS = {
    "WORKERS": -1,
    "MIN_LENGTH": 100,
    "FRAME_LENGTH": 100,
    "MIN_IDENTITY": "0.9",
    "MIN_END": 10,
    "ANCHOR_SIZE": 20,
    "ANCHOR_FP": "0.1",
    "MAX_ANCHOR_FRAGMENTS": 100000,
    "ALIGNER": "similar",
    "MISMATCH_CHECK": 1,
    "GAP_CHECK": 2,
    "ALIGNED_CHECK": 10,
    "MAX_TAIL": 3,           # CMakeLists.txt:89 (MoveGaps)
    "MAX_TAIL_TO_GAP": "1.0",  # CMakeLists.txt:90 (MoveGaps)
}


class Decimal:
    """4-digit fixed point (src/util/Decimal.hpp:25-213): value = impl / 10000."""

    SUB = 10000

    def __init__(self, value=0):
        if isinstance(value, Decimal):
            self.impl = value.impl
        elif isinstance(value, int):
            self.impl = value * self.SUB
        elif isinstance(value, float):
            self.impl = Decimal(repr(value)).impl
        else:
            s = str(value)
            if "." in s:
                ip, fr = s.split(".", 1)
                i = int(ip) if ip not in ("", "-") else 0
                j = int((fr + "0000")[:4])
                if s.startswith("-"):
                    j = -j
                self.impl = i * self.SUB + j
            else:
                self.impl = int(s) * self.SUB

    @classmethod
    def raw(cls, impl):
        d = cls()
        d.impl = impl
        return d

    def to_d(self):
        return self.impl / float(self.SUB)

    def to_i(self):
        return self.impl // self.SUB if self.impl >= 0 else -((-self.impl) // self.SUB)

    def __mul__(self, o):
        o = o if isinstance(o, Decimal) else Decimal(o)
        v = self.impl * o.impl
        q = abs(v) // self.SUB
        return Decimal.raw(q if v >= 0 else -q)

    def __repr__(self):
        return "Decimal(%s)" % (self.impl / self.SUB)


class OptionError(ValueError):
    pass


class Processor:
    """Base of all hot-path processors (Processor.hpp:42-510, subset)."""

    name = "Processor"

    def __init__(self):
        self._opts = {}       # name -> [value, type, description]
        self._ignored = set()
        self._rules = []      # (text, predicate)
        self._bs = {"target": BlockSet(), "other": BlockSet()}
        self._workers = -1
        self.timing = []      # [(stage, ms)] of the last run

    # -- options ------------------------------------------------------------
    def add_opt(self, name, description, default, typ=None):
        typ = typ or (bool if isinstance(default, bool) else int if isinstance(default, int)
                      else Decimal if isinstance(default, Decimal) else str)
        self._opts[name] = [self._convert(default, typ), typ, description]

    def add_gopt(self, name, description, global_name, typ=None):
        default = GLOBAL_OPTS[global_name]
        self.add_opt(name, description, default, typ or type(default))

    def add_opt_rule(self, text, pred):
        self._rules.append((text, pred))

    @staticmethod
    def _convert(v, typ):
        if typ is bool:
            if isinstance(v, str):
                return v.lower() in ("1", "true", "yes")
            return bool(v)
        if typ is int:
            return int(v)
        if typ is Decimal:
            return Decimal(v)
        return v

    def has_opt(self, name):
        return name in self._opts

    def opt_value(self, name):
        return self._opts[name][0]

    def set_opt_value(self, name, value):
        if name not in self._opts:
            raise OptionError("Unknown option %s of %s" % (name, self.name))
        if name in self._ignored:
            return
        self._opts[name][0] = self._convert(value, self._opts[name][1])

    def add_ignored_option(self, name):
        self._ignored.add(name)

    def set_options(self, options, bs_source=None):
        """Option string grammar of Processor::set_options (Processor.cpp:260-322):
        ``--opt=v`` sets, ``--opt:=v`` sets and fixes, ``target=name`` maps a
        block set (resolved through ``bs_source``, a dict name -> BlockSet),
        ``no_options`` and ``prefix|...`` are accepted."""
        fixed = []
        for tok in shlex.split(options or ""):
            tok = tok.rstrip()
            if "=" in tok:
                eq = tok.index("=")
                if tok.startswith("-"):
                    name, val = tok[:eq], tok[eq + 1:]
                    ignore = name.endswith(":")
                    if ignore:
                        name = name[:-1]
                    short = name[2:] if name.startswith("--") else name[1:]
                    self.set_opt_value(short, val)
                    if ignore:
                        fixed.append(short)
                elif bs_source is not None:
                    mine, theirs = tok[:eq], tok[eq + 1:]
                    self._bs[mine] = bs_source.setdefault(theirs, BlockSet())
            elif tok == "no_options" or tok.startswith("prefix|"):
                pass
        for name in fixed:
            self.add_ignored_option(name)

    def set_workers(self, w):
        self._workers = w

    def workers(self):
        return self._workers

    # -- block sets ---------------------------------------------------------
    def set_bs(self, name, bs):
        self._bs[name] = bs

    def get_bs(self, name):
        return self._bs.setdefault(name, BlockSet())

    def block_set(self):
        return self._bs["target"]

    def set_block_set(self, bs):
        self._bs["target"] = bs

    def other(self):
        return self._bs["other"]

    # -- running ------------------------------------------------------------
    def check_options(self):
        for text, pred in self._rules:
            if not pred(self):
                raise OptionError("Option rule failed: " + text)

    def run(self):
        """Processor::run (Processor.cpp:652-673): check options, run_impl()."""
        self.check_options()
        self.run_impl()

    def apply(self, bs):
        """Processor::apply: run with ``bs`` as target."""
        old = self._bs.get("target")
        self._bs["target"] = bs
        try:
            self.run()
        finally:
            self._bs["target"] = old

    def run_impl(self):
        raise NotImplementedError


_REGISTRY = {}


def register(cls):
    """Meta::set_processor<T> (src/algo/Meta.hpp:84-87, meta_lib.cpp:101-195)."""
    _REGISTRY[cls.name] = cls
    return cls


def new_p(name):
    """lua_lib.lua:59-61 new_p."""
    try:
        return _REGISTRY[name]()
    except KeyError:
        raise OptionError("Unknown processor: " + name)


def processors():
    return sorted(_REGISTRY)


def run(name, opts="", blocksets=None):
    """lua_lib.lua:128-133 run(name, opts): new processor, apply options, run."""
    p = new_p(name)
    if isinstance(opts, dict):
        for k, v in opts.items():
            if isinstance(v, BlockSet):
                p.set_bs(k, v)
            else:
                p.set_opt_value(k.replace("_", "-"), v)
    else:
        p.set_options(opts, blocksets)
    p.run()
    return p
