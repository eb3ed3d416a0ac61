"""Small concurrency helpers of the parallel package (reference deeplearning4j-core/src/main/java/org/deeplearning4j/
parallelism/MultiBoolean.java and AsyncIterator.java).

MultiBoolean: a fixed set of flags with all-true / all-false queries. In one-time mode the set freezes as soon as
every flag has left its initial value, so late updates from workers that already finished cannot flip it back.

AsyncIterator: wraps any iterator with a daemon producer thread and a bounded queue (``bufferSize``), so a slow
source (record parsing, decompression) runs ahead of the consumer; the end is a sentinel, and a producer exception is
re-raised in the consumer."""
import queue
import threading


class MultiBoolean:
    def __init__(self, numEntries, initialValue=False, oneTime=False):
        if numEntries < 1:
            raise ValueError("MultiBoolean needs at least one entry")
        self.n, self.initial, self.oneTime = int(numEntries), bool(initialValue), bool(oneTime)
        self.bits = [self.initial] * self.n
        self._frozen = False
        self._lock = threading.Lock()

    def set(self, value, entry):
        if not 0 <= entry < self.n:
            raise IndexError(f"entry {entry} out of range [0, {self.n})")
        with self._lock:
            if self._frozen:
                return
            self.bits[entry] = bool(value)
            if self.oneTime and all(b != self.initial for b in self.bits):
                self._frozen = True

    def get(self, entry):
        return self.bits[entry]

    def allTrue(self):
        with self._lock:
            return all(self.bits)

    def allFalse(self):
        with self._lock:
            return not any(self.bits)


class AsyncIterator:
    _END = object()

    def __init__(self, iterator, bufferSize=1024):
        self._q = queue.Queue(maxsize=max(1, int(bufferSize)))
        self._next = None
        self._done = False
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, args=(iter(iterator),), daemon=True)
        self._t.start()

    def _run(self, it):
        try:
            for v in it:
                while not self._stop.is_set():
                    try:
                        self._q.put(("v", v), timeout=0.1)
                        break
                    except queue.Full:
                        continue
                if self._stop.is_set():
                    return
            self._q.put(("end", None))
        except BaseException as e:          # surfaced in the consumer
            self._q.put(("err", e))

    def hasNext(self):
        if self._done:
            return False
        if self._next is None:
            kind, v = self._q.get()
            if kind == "end":
                self._done = True
                return False
            if kind == "err":
                self._done = True
                raise v
            self._next = (v,)
        return True

    def next(self):
        if not self.hasNext():
            raise StopIteration
        v = self._next[0]
        self._next = None
        return v

    def __iter__(self):
        return self

    __next__ = next

    def shutdown(self):
        self._stop.set()
        self._done = True
