"""Plain (non-encoded) gradient sharing between the worker threads of one process, and the broadcast queue the
reference's accumulators use to fan messages out to every consumer.

Reference:
  * NN:optimize/solvers/accumulation/BasicGradientsAccumulator.java:26-157 — ``storeUpdate`` (barrier, the first
    thread sums every party's candidate into ``storage`` and hands it to the MessageHandler), ``receiveUpdate``
    (``updates += array`` under the write lock), ``applyUpdate(function, params, grad[, alpha])`` (every thread steps
    its params by ``updates``, barrier, the first one clears ``updates``, barrier), ``reset``.
  * NN:optimize/solvers/accumulation/LocalHandler.java — the MessageHandler that loops ``broadcastUpdates`` straight
    back into the same accumulator's ``receiveUpdate``.
  * NN:optimize/solvers/accumulation/FancyBlockingQueue.java — a BlockingQueue where each of ``consumers`` threads
    sees EVERY element once (the head is removed only after all consumers have taken it), with ``registerConsumers``
    fixing the number of elements ready for this round and ``fallbackToSingleConsumerMode`` turning it into a plain
    queue. Tests: deeplearning4j-core/.../parallelism/FancyBlockingQueueTests.java.

Design here: the accumulator is one object shared by the in-process ParallelWrapper's worker threads (one replica per
GPU, parallel/inprocess.py, TrainingMode.CUSTOM). Candidates live on their workers' devices; the first thread sums
them into a device-resident ``storage`` on its own device (device-to-device copies over xGMI for the other
replicas' arrays), and every thread applies ``updates`` to its own parameters, copied to its device. The per-step
network hook ``apply_update`` computes the worker's post-updater update with the fused updater (parameters left
untouched), shares it, and steps the parameters by the sum of all parties' updates — so N replicas stay identical and
the step equals N workers' updates summed (the reference's semantics; the updater state stays per replica).
The queue uses per-consumer cursors under one condition variable instead of the reference's spin barriers: same
observable contract (every consumer sees every element in FIFO order; an element is dropped once all consumers took
it), no busy waiting.
"""
import itertools
import threading

import torch

_tokens = itertools.count()


class FancyBlockingQueue:
    """Broadcast FIFO: ``registerConsumers(n)`` consumers each receive every element once, in order.

    ``put/add/offer`` append; ``poll()`` returns the calling consumer's next element (None when it has drained what
    is ready); ``isEmpty()`` is per consumer: True once it has taken every element that was ready at
    ``registerConsumers`` time (or since, for elements put later). ``fallbackToSingleConsumerMode(True)`` makes it a
    plain queue (each element to one consumer)."""

    def __init__(self, capacity=0, consumers=-1):
        self.capacity = int(capacity)
        self._items = []                 # elements not yet taken by every consumer
        self._base = 0                   # absolute index of _items[0]
        self._cursor = {}                # consumer thread id -> absolute index of its next element
        self._consumers = int(consumers)
        self._bypass = False
        self._cv = threading.Condition()
        self._local = threading.local()  # per-thread consumer token (thread idents are recycled after exit)

    # ----------------------------------------------------------------------------------------------- producers
    def put(self, e, timeout=None):
        with self._cv:
            if self.capacity > 0:
                if not self._cv.wait_for(lambda: len(self._items) < self.capacity, timeout):
                    raise TimeoutError("FancyBlockingQueue full")
            self._items.append(e)
            self._cv.notify_all()

    def add(self, e):
        with self._cv:
            if self.capacity > 0 and len(self._items) >= self.capacity:
                raise OverflowError("FancyBlockingQueue full")
            self._items.append(e)
            self._cv.notify_all()
        return True

    def offer(self, e):
        with self._cv:
            if self.capacity > 0 and len(self._items) >= self.capacity:
                return False
            self._items.append(e)
            self._cv.notify_all()
        return True

    # ----------------------------------------------------------------------------------------------- consumers
    def registerConsumers(self, consumers):
        with self._cv:
            self._consumers = int(consumers)
            self._cursor = {}

    def fallbackToSingleConsumerMode(self, really=True):
        with self._cv:
            self._bypass = bool(really)

    def _me(self):
        tid = getattr(self._local, "token", None)
        if tid is None:
            tid = self._local.token = next(_tokens)
        cur = self._cursor.get(tid)
        if cur is None:
            if self._consumers > 0 and len(self._cursor) >= self._consumers:
                raise RuntimeError(f"FancyBlockingQueue: more than {self._consumers} registered consumers")
            cur = self._cursor[tid] = self._base
        return tid, cur

    def _trim(self):
        if not self._cursor or self._consumers <= 0 or len(self._cursor) < self._consumers:
            return
        low = min(self._cursor.values())
        drop = low - self._base
        if drop > 0:
            del self._items[:drop]
            self._base = low
            self._cv.notify_all()

    def poll(self, timeout=None):
        with self._cv:
            if self._bypass or self._consumers <= 1:
                if timeout and not self._items:
                    self._cv.wait_for(lambda: self._items, timeout)
                if not self._items:
                    return None
                self._base += 1
                e = self._items.pop(0)
                self._cv.notify_all()
                return e
            tid, cur = self._me()
            if timeout:
                self._cv.wait_for(lambda: self._cursor[tid] - self._base < len(self._items), timeout)
                cur = self._cursor[tid]
            if cur - self._base >= len(self._items):
                return None
            e = self._items[cur - self._base]
            self._cursor[tid] = cur + 1
            self._trim()
            return e

    def isEmpty(self):
        with self._cv:
            if self._bypass or self._consumers <= 1:
                return not self._items
            tid, cur = self._me()
            return cur - self._base >= len(self._items)

    def peek(self):
        with self._cv:
            return self._items[0] if self._items else None

    def size(self):
        with self._cv:
            return len(self._items)

    def clear(self):
        with self._cv:
            self._base += len(self._items)
            self._items = []
            for k in self._cursor:
                self._cursor[k] = self._base
            self._cv.notify_all()

    def __len__(self):
        return self.size()


class LocalHandler:
    """MessageHandler that delivers ``broadcastUpdates`` to the accumulator it was initialised with."""

    def __init__(self):
        self.accumulator = None

    def initialize(self, accumulator):
        self.accumulator = accumulator

    def broadcastUpdates(self, updates):
        self.accumulator.receiveUpdate(updates)
        return True


class BasicGradientsAccumulator:
    """The reference's plain GradientsAccumulator for ``parties`` worker threads of one process (see module doc).

    Used as a ParallelWrapper CUSTOM accumulator: ``ParallelWrapper.Builder(net).workers(n).inProcess(True)
    .gradientsAccumulator(BasicGradientsAccumulator(n))`` shares ONE instance between the n replicas."""
    handles_update = True
    shared_in_process = True             # the in-process wrapper gives every replica this same instance

    def __init__(self, parties, handler=None, timeout=600.0):
        self.parties = int(parties)
        self.handler = handler if handler is not None else LocalHandler()
        self.handler.initialize(self)
        self.storage = None
        self.updates = None
        self.ownCounter = 0
        self.extCounter = 0
        self._has = False
        self._candidates = [None] * self.parties
        self._slot = {}
        self._local = threading.local()
        self._slot_lock = threading.Lock()
        self._lock = threading.RLock()
        self._timeout = timeout
        self._barrier = threading.Barrier(self.parties, timeout=timeout)

    def _party(self):
        tid = getattr(self._local, "token", None)
        if tid is None:
            tid = self._local.token = next(_tokens)
        with self._slot_lock:
            s = self._slot.get(tid)
            if s is None:
                if len(self._slot) >= self.parties:
                    raise RuntimeError(f"BasicGradientsAccumulator: more than {self.parties} parties")
                s = self._slot[tid] = len(self._slot)
            return s

    def resetParties(self):
        """Forget which threads are the parties (a new set of worker threads is about to start)."""
        with self._slot_lock:
            self._slot = {}
            self._local = threading.local()
            self._candidates = [None] * self.parties
            self._barrier.reset()

    def abort(self):
        """Break the barriers (a failing worker): every waiting party raises instead of hanging."""
        self._barrier.abort()

    # ------------------------------------------------------------------------------------------- reference SPI
    def storeUpdate(self, array):
        """Contribute this party's update; after the barrier the first party sums all candidates into ``storage``
        and broadcasts it through the handler (into ``updates`` for the LocalHandler)."""
        me = self._party()
        if array.is_cuda:
            torch.cuda.current_stream(array.device).synchronize()   # the candidate is read from another thread
        self._candidates[me] = array
        if self._barrier.wait() == 0:
            first = self._candidates[0]
            if self.storage is None or self.storage.shape != first.shape or self.storage.device != first.device:
                self.storage = torch.zeros_like(first)
            else:
                self.storage.zero_()
            for c in self._candidates:
                self.storage.add_(c.to(self.storage.device, non_blocking=False))
            if self.storage.is_cuda:
                torch.cuda.current_stream(self.storage.device).synchronize()
            if self.handler.broadcastUpdates(self.storage):
                self.ownCounter += 1
            self._candidates = [None] * self.parties
        self._barrier.wait()

    def receiveUpdate(self, array):
        with self._lock:
            self.extCounter += 1
            if self.updates is None or self.updates.shape != array.shape:
                self.updates = torch.zeros_like(array)
            self.updates.add_(array.to(self.updates.device))
            if self.updates.is_cuda:
                torch.cuda.current_stream(self.updates.device).synchronize()
            self._has = True

    def applyUpdate(self, function, params, grad=None, alpha=None):
        """Every party steps its ``params`` by the shared ``updates`` (``function.step(params, updates[, alpha])``);
        then the first party clears them."""
        if self._has and self.updates is not None:
            u = self.updates.to(params.device)
            if alpha is None:
                function.step(params, u)
            else:
                function.step(params, u, alpha)
            if params.is_cuda:
                torch.cuda.current_stream(params.device).synchronize()
        if self._barrier.wait() == 0:
            if self.updates is not None:
                self.updates.zero_()
            self._has = False
        self._barrier.wait()

    def reset(self):
        with self._lock:
            if self.storage is not None:
                self.storage.zero_()
            if self.updates is not None:
                self.updates.zero_()
            self._has = False

    def touch(self):
        pass

    def setExternalSource(self, source):
        raise NotImplementedError("BasicGradientsAccumulator has no external source (reference: "
                                  "UnsupportedOperationException)")

    # ------------------------------------------------------------------------------------------- network hook
    def begin_backward(self, net):
        pass

    def grad_ready(self, net, offset):
        pass

    def reduce_gradients(self, net):
        pass

    def apply_update(self, net, batch_size, iteration, epoch):
        """One worker step: post-updater update u of this replica (fused updater; parameters restored), shared with
        storeUpdate, then params -= sum over parties of u (NegativeGradientStepFunction)."""
        from ..optimize.solvers import NegativeGradientStepFunction
        p, g = net.flattenedParams, net.flattenedGradients
        keep = p.clone()
        net.updater.update(p, g, iteration, epoch, batch_size)     # g <- update (p stepped, restored below)
        p.copy_(keep)
        self.storeUpdate(g.clone())
        self.applyUpdate(NegativeGradientStepFunction(), p, g)
        net.sync_shadow()

    def idle_step(self, net):
        """A replica with no batch in a trailing partial round: contributes a zero update and applies the others'."""
        from ..optimize.solvers import NegativeGradientStepFunction
        p = net.flattenedParams
        self.storeUpdate(torch.zeros_like(p))
        self.applyUpdate(NegativeGradientStepFunction(), p)
        net.sync_shadow()
