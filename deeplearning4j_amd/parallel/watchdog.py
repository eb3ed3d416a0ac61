"""Failure detection, fault injection and recovery.

Reference behaviour: worker exceptions are stored and rethrown to the master (PW:trainer/DefaultTrainer.java:
396-416); an ``AtomicThrowable`` poisons spinning threads (EncodedGradientsAccumulator.java:59,168-170);
``InvalidScoreIterationTerminationCondition`` stops on NaN scores; ``SleepyTrainingListener`` injects latency;
there is no elasticity — recovery is "restart from the last checkpoint".

MI355X-native equivalents (one process per GPU, RCCL):
* :class:`StepWatchdog` — a heartbeat per training iteration; when a step (typically a hung collective on a dead
  peer) exceeds its deadline the watchdog dumps every thread's stack and aborts the process, so the launcher
  tears the job down instead of hanging 8 GPUs. RCCL's own async error handling is switched on by
  :func:`deeplearning4j_amd.parallel.distributed.init_distributed` (``TORCH_NCCL_ASYNC_ERROR_HANDLING``).
* :class:`NaNGuardListener` — finite-score check every N iterations (one host sync per check, not per step).
* :class:`FaultInjectionListener` — deterministic failures / stalls at a chosen iteration (and rank) for tests.
* :func:`fit_with_recovery` — run a training function; on failure reload the last checkpoint written by
  :class:`~deeplearning4j_amd.optimize.listeners.CheckpointListener` and continue, up to ``maxRestarts`` times.
"""
import faulthandler
import logging
import math
import os
import sys
import threading
import time

log = logging.getLogger(__name__)


class InvalidScoreException(RuntimeError):
    pass


class InjectedFault(RuntimeError):
    pass


class StepWatchdog:
    """``heartbeat()`` once per step (or attach as a listener). If no heartbeat arrives within ``timeout_s`` the
    ``action`` runs: "abort" (dump stacks, ``os._exit(exit_code)``), "raise" (the next heartbeat raises), or a
    callable(watchdog)."""

    def __init__(self, timeout_s=300.0, action="abort", exit_code=75, poll_s=None):
        self.timeout_s = float(timeout_s)
        self.action = action
        self.exit_code = int(exit_code)
        self.poll_s = poll_s or max(0.05, min(5.0, self.timeout_s / 10))
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._fired = False
        self._lock = threading.Lock()
        self._t = threading.Thread(target=self._run, name="dl4j-step-watchdog", daemon=True)
        self._t.start()

    def heartbeat(self):
        with self._lock:
            self._last = time.monotonic()
            fired = self._fired
        if fired and self.action == "raise":
            raise TimeoutError(f"training step exceeded the {self.timeout_s}s watchdog deadline")

    # listener SPI
    def iterationDone(self, model, iteration, epoch):
        self.heartbeat()

    def _run(self):
        while not self._stop.wait(self.poll_s):
            with self._lock:
                late = time.monotonic() - self._last > self.timeout_s and not self._fired
                if late:
                    self._fired = True
            if late:
                self._fire()

    def _fire(self):
        msg = f"[watchdog] no training-step heartbeat for {self.timeout_s}s (pid {os.getpid()})"
        log.error(msg)
        print(msg, file=sys.stderr, flush=True)
        if self.action == "abort":
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
            sys.stderr.flush()
            os._exit(self.exit_code)
        elif callable(self.action):
            self.action(self)

    def fired(self):
        return self._fired

    def close(self):
        self._stop.set()
        self._t.join(timeout=1.0)


class NaNGuardListener:
    """Raise (or call ``onInvalid``) when the score is NaN/Inf. Checks every ``frequency`` iterations."""

    def __init__(self, frequency=1, onInvalid=None):
        self.frequency = max(1, int(frequency))
        self.onInvalid = onInvalid

    def iterationDone(self, model, iteration, epoch):
        if iteration % self.frequency:
            return
        s = model.score()
        if s is None or not math.isfinite(s):
            if self.onInvalid is not None:
                self.onInvalid(model, iteration, s)
            else:
                raise InvalidScoreException(f"invalid score {s} at iteration {iteration}")


class FaultInjectionListener:
    """Inject a failure (exception) or a stall (sleep) at ``atIteration``, optionally only on one rank."""

    def __init__(self, atIteration, mode="raise", sleepMs=0, rank=None, once=True):
        self.atIteration = int(atIteration)
        self.mode = mode
        self.sleepMs = int(sleepMs)
        self.rank = rank
        self.once = once
        self.triggered = 0

    def iterationDone(self, model, iteration, epoch):
        if iteration != self.atIteration or (self.once and self.triggered):
            return
        if self.rank is not None and int(os.environ.get("RANK", "0")) != int(self.rank):
            return
        self.triggered += 1
        if self.mode == "sleep":
            time.sleep(self.sleepMs / 1000.0)
        else:
            raise InjectedFault(f"injected fault at iteration {iteration}")


def fit_with_recovery(model, train_fn, checkpointListener, maxRestarts=3, device=None):
    """``train_fn(model)`` runs training (with ``checkpointListener`` attached). On an exception the last
    checkpoint is restored (params, updater state, iteration/epoch counters) and ``train_fn`` is called again on the
    restored model. Returns (model, restarts)."""
    restarts = 0
    while True:
        try:
            train_fn(model)
            return model, restarts
        except (KeyboardInterrupt, SystemExit):
            raise
        except Exception as e:  # noqa: BLE001 - any worker failure triggers the restart path
            if restarts >= maxRestarts:
                raise
            last = checkpointListener.lastCheckpoint()
            if last is None:
                raise
            log.warning("training failed (%s); restoring checkpoint %s", e, last.checkpointNum)
            restored = checkpointListener.loadCheckpoint(last, True, device or getattr(model, "device", None))
            restored.setListeners(model.getListeners())
            model = restored
            restarts += 1
