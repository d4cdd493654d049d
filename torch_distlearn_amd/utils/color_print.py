"""Coloured protocol logging (lua/colorPrint.lua:1-17).

``printServer`` prints red, ``printClient(node, s)`` prints blue with a
"Client #n" prefix; non-strings are printed raw.  Unlike the reference these
are module functions (not globals) and they can be silenced with
:func:`set_verbose` (the reference scripts redefine the globals to no-ops when
``--verbose`` is off, examples/EASGD_server.lua:51-56).
"""
from __future__ import annotations

import sys

_RED = "\x1b[31m"
_BLUE = "\x1b[34m"
_RESET = "\x1b[0m"
_VERBOSE = True


def set_verbose(flag: bool) -> None:
    global _VERBOSE
    _VERBOSE = bool(flag)


def _color_ok() -> bool:
    return sys.stdout.isatty()


def printServer(string) -> None:  # noqa: N802 (reference API name)
    if not _VERBOSE:
        return
    if isinstance(string, str):
        print(f"{_RED}{string}{_RESET}" if _color_ok() else string, flush=True)
    else:
        print(string, flush=True)


def printClient(node, string) -> None:  # noqa: N802
    if not _VERBOSE:
        return
    if isinstance(string, str):
        msg = f"Client #{node} {string}"
        print(f"{_BLUE}{msg}{_RESET}" if _color_ok() else msg, flush=True)
    else:
        print(string, flush=True)


print_server = printServer
print_client = printClient
