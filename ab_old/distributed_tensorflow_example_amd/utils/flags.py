"""tf.app.flags-compatible command-line flags (example.py:33-35; lr2.py:17-35).

`DEFINE_string/integer/float/boolean/bool/list/enum`, a global `FLAGS` parsed
lazily on first attribute access (unknown argv entries are left for the
program), attribute assignment for ad-hoc config (`FLAGS.work_dir = ...`,
model_export.py:10-11), `--flag=value`, `--flag value`, `--[no]bool`, and
`app.run(main)`.  Built on argparse; also used by the Python launcher that
replaces the vendored shflags scripts.
"""
from __future__ import annotations

import argparse
import sys
from typing import Any, Dict, List, Optional


def _str2bool(v):
    if isinstance(v, bool):
        return v
    if v.lower() in ("1", "true", "t", "yes", "y"):
        return True
    if v.lower() in ("0", "false", "f", "no", "n"):
        return False
    raise argparse.ArgumentTypeError(f"not a boolean: {v}")


class _FlagValues:
    def __init__(self):
        object.__setattr__(self, "_defs", {})
        object.__setattr__(self, "_values", {})
        object.__setattr__(self, "_parsed", False)
        object.__setattr__(self, "_remaining", [])

    # ---------------------------------------------------------------- defining
    def _define(self, name, default, help_, kind, **extra):
        self._defs[name] = dict(default=default, help=help_, kind=kind, **extra)
        if name not in self._values:
            self._values[name] = default

    # ---------------------------------------------------------------- parsing
    def _parser(self):
        p = argparse.ArgumentParser(add_help=True, allow_abbrev=False)
        for name, d in self._defs.items():
            k = d["kind"]
            if k == "bool":
                p.add_argument(f"--{name}", default=d["default"], type=_str2bool, help=d["help"])
                p.add_argument(f"--no{name}", dest=name, action="store_false")
            elif k == "list":
                p.add_argument(f"--{name}", default=d["default"],
                               type=lambda s: [x for x in s.split(",") if x], help=d["help"])
            elif k == "enum":
                p.add_argument(f"--{name}", default=d["default"], choices=d["enum_values"], help=d["help"])
            else:
                p.add_argument(f"--{name}", default=d["default"], type={"string": str, "integer": int,
                                                                        "float": float}[k], help=d["help"])
        return p

    def __call__(self, argv: Optional[List[str]] = None, known_only: bool = True) -> List[str]:
        argv = list(sys.argv if argv is None else argv)
        prog, args = argv[:1], argv[1:]
        # gflags booleans: bare `--flag` means true and never consumes the next word
        bools = {n for n, d in self._defs.items() if d["kind"] == "bool"}
        args = [f"{a}=true" if a.startswith("--") and a[2:] in bools else a for a in args]
        ns, rest = self._parser().parse_known_args(args)
        for k, v in vars(ns).items():
            self._values[k] = v
        object.__setattr__(self, "_parsed", True)
        object.__setattr__(self, "_remaining", rest)
        return prog + rest

    def _ensure(self):
        if not self._parsed:
            try:
                self(sys.argv)
            except SystemExit:
                raise

    def mark_as_parsed(self):
        object.__setattr__(self, "_parsed", True)

    def reset(self):
        self._values.clear()
        for k, d in self._defs.items():
            self._values[k] = d["default"]
        object.__setattr__(self, "_parsed", False)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        if name in self._defs:
            self._ensure()
        if name in self._values:
            return self._values[name]
        raise AttributeError(f"Unknown flag --{name}")

    def __setattr__(self, name, value):
        self._values[name] = value

    def __contains__(self, name):
        return name in self._values

    def flag_values_dict(self) -> Dict[str, Any]:
        self._ensure()
        return dict(self._values)

    def get(self, name, default=None):
        return self._values.get(name, default)


FLAGS = _FlagValues()


def DEFINE_string(name, default, help="", flag_values=FLAGS):  # noqa: N802,A002
    flag_values._define(name, default, help, "string")


def DEFINE_integer(name, default, help="", flag_values=FLAGS, lower_bound=None, upper_bound=None):  # noqa: N802
    flag_values._define(name, default, help, "integer")


def DEFINE_float(name, default, help="", flag_values=FLAGS):  # noqa: N802
    flag_values._define(name, default, help, "float")


def DEFINE_boolean(name, default, help="", flag_values=FLAGS):  # noqa: N802
    flag_values._define(name, default, help, "bool")


DEFINE_bool = DEFINE_boolean


def DEFINE_list(name, default, help="", flag_values=FLAGS):  # noqa: N802
    if isinstance(default, str):
        default = [x for x in default.split(",") if x]
    flag_values._define(name, default, help, "list")


def DEFINE_enum(name, default, enum_values, help="", flag_values=FLAGS):  # noqa: N802
    flag_values._define(name, default, help, "enum", enum_values=list(enum_values))


def run(main=None, argv=None):
    """tf.app.run: parse flags, call main(remaining_argv), exit with its code."""
    remaining = FLAGS(argv if argv is not None else sys.argv)
    main = main or sys.modules["__main__"].main
    sys.exit(main(remaining))
