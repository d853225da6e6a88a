"""Bounded failure for multi-rank setup (no counterpart in the reference, whose destructor
barrier hangs every peer of a rank that fails, tensor_p2p_cache.cc:115).

A rank that stalls in a setup collective -- process-group rendezvous, the RCCL communicator,
the IPC-handle exchange of TensorP2PServer / the services, a self-check -- would otherwise hold
every other rank (and the job's lease) until an outer time limit.  SetupWatchdog names the step
a rank is in; when a step outlives its bound, a daemon thread prints the rank, the step and the
elapsed time to stderr and ends the process with os._exit(code) (no exec, no cleanup that could
block on the stalled collective).  Each rank runs its own, so every rank of a stalled setup
exits non-zero within the bound, whichever rank withheld the collective."""
import os
import sys
import threading
import time

__all__ = ["SetupWatchdog"]


class SetupWatchdog:
    def __init__(self, seconds=600.0, rank=None, what="setup", exit_code=3, poll=0.2):
        self.default = float(seconds)
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else int(rank)
        self.what, self.exit_code, self.poll = what, int(exit_code), float(poll)
        self._lock = threading.Lock()
        self._step, self._t0, self._bound = None, 0.0, 0.0
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="dgs-setup-watchdog",
                                        daemon=True)
        self._thread.start()

    def step(self, name, seconds=None):
        """Enter step `name`, bounded by `seconds` (default: the watchdog's bound)."""
        with self._lock:
            self._step, self._t0 = name, time.monotonic()
            self._bound = self.default if seconds is None else float(seconds)
        return self

    def done(self):
        """Setup finished: disarm (the thread ends)."""
        with self._lock:
            self._step = None
        self._stop.set()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.done()
        return False

    def _run(self):
        while not self._stop.wait(self.poll):
            with self._lock:
                step, t0, bound = self._step, self._t0, self._bound
            if step is None:
                continue
            el = time.monotonic() - t0
            if el > bound:
                sys.stderr.write(f"[dgs watchdog] rank {self.rank}: {self.what} step '{step}' "
                                 f"did not finish within {bound:.0f} s ({el:.1f} s); exiting "
                                 f"with status {self.exit_code}\n")
                sys.stderr.flush()
                os._exit(self.exit_code)
