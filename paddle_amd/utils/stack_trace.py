"""Per-thread stack of the operators (or layers) being executed, dumped when an op
fails or on demand (reference paddle/legacy/utils/CustomStackTrace: the layer
stack printed on a fatal signal).  ``install()`` turns it on: the executor pushes
each op, an exception raised inside an op carries the stack in its message,
``SIGUSR1`` prints every thread's stack, and ``faulthandler`` prints the Python
stacks on SIGSEGV / SIGABRT."""
from __future__ import annotations

import contextlib
import faulthandler
import signal
import sys
import threading

_tls = threading.local()
_all: dict[int, list] = {}
enabled = [False]


def _stack():
    s = getattr(_tls, "stack", None)
    if s is None:
        s = _tls.stack = []
        _all[threading.get_ident()] = s
    return s


@contextlib.contextmanager
def frame(name):
    """Push ``name`` while the block runs; on an exception, record the stack."""
    s = _stack()
    s.append(name)
    try:
        yield
    except Exception as e:
        if not getattr(e, "_pa_op_stack", None):
            try:
                e._pa_op_stack = list(s)
                e.add_note(f"operator stack (outermost first): {' -> '.join(s)}")
            except (AttributeError, TypeError):  # exceptions without notes (py < 3.11) keep the attribute
                pass
        raise
    finally:
        s.pop()


def current():
    return list(_stack())


def dump(file=None):
    f = file or sys.stderr
    for tid, s in list(_all.items()):
        print(f"thread {tid}: {' -> '.join(s) if s else '(idle)'}", file=f, flush=True)


def install(sig=signal.SIGUSR1):
    enabled[0] = True
    faulthandler.enable(all_threads=True)
    if threading.current_thread() is threading.main_thread():
        signal.signal(sig, lambda *_: dump())


def uninstall():
    enabled[0] = False
