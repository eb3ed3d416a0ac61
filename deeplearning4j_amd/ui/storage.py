"""Stats storage: the Persistable record model, routers and stores.

Reference: CORE:api/storage/{StatsStorage, StatsStorageRouter, Persistable, StorageMetaData, StatsStorageListener,
StatsStorageEvent}.java; implementations InMemoryStatsStorage, FileStatsStorage (MapDB) / J7FileStatsStorage (SQLite),
RemoteUIStatsStorageRouter (HTTP POST to a remote UI), CollectionStatsStorageRouter.
Records are JSON documents here (the reference's SBE binary encoding is a JVM detail); the SQLite store keeps one
table per record kind keyed by (session, type, worker, timestamp), like J7FileStatsStorage.
"""
import json
import sqlite3
import threading
import time
import urllib.request


class Persistable:
    """A storable record: identity (session/type/worker/timestamp) + a JSON payload."""

    def __init__(self, sessionID="", typeID="", workerID="", timeStamp=None, data=None, kind="update"):
        self.sessionID, self.typeID, self.workerID = sessionID, typeID, workerID
        self.timeStamp = int(time.time() * 1000) if timeStamp is None else int(timeStamp)
        self.data = dict(data or {})
        self.kind = kind

    def getSessionID(self):
        return self.sessionID

    def getTypeID(self):
        return self.typeID

    def getWorkerID(self):
        return self.workerID

    def getTimeStamp(self):
        return self.timeStamp

    def to_dict(self):
        return {"sessionID": self.sessionID, "typeID": self.typeID, "workerID": self.workerID,
                "timeStamp": self.timeStamp, "kind": self.kind, "data": self.data}

    def encode(self):
        return json.dumps(self.to_dict()).encode("utf-8")

    def encodingLengthBytes(self):
        return len(self.encode())

    @staticmethod
    def decode(b):
        d = json.loads(b.decode("utf-8") if isinstance(b, (bytes, bytearray)) else b)
        return Persistable(d["sessionID"], d["typeID"], d["workerID"], d["timeStamp"], d["data"], d.get("kind"))

    def __getitem__(self, k):
        return self.data[k]

    def get(self, k, default=None):
        return self.data.get(k, default)

    def __repr__(self):
        return f"Persistable({self.kind}, {self.sessionID}/{self.typeID}/{self.workerID}@{self.timeStamp})"


class StorageMetaData(Persistable):
    """Session metadata: the record classes used for initialisation / updates plus optional extra metadata (a JSON
    value here; the reference's SbeStorageMetaData carries a Java-serialised object)."""

    def __init__(self, sessionID=None, typeID=None, workerID="", initTypeClass=None, updateTypeClass=None,
                 timeStamp=None, extraMeta=None):
        super().__init__(sessionID, typeID, workerID, 0 if timeStamp is None and sessionID is None else timeStamp,
                         {"initTypeClass": initTypeClass, "updateTypeClass": updateTypeClass,
                          "extraMeta": extraMeta}, "meta")

    def getInitTypeClass(self):
        return self.data.get("initTypeClass")

    def getUpdateTypeClass(self):
        return self.data.get("updateTypeClass")

    def getExtraMetaData(self):
        return self.data.get("extraMeta")

    def decode(self, b):
        """In place, as the reference's ``m2.decode(bytes)``; also returns self."""
        d = json.loads(b.decode("utf-8") if isinstance(b, (bytes, bytearray)) else b)
        self.sessionID, self.typeID, self.workerID = d["sessionID"], d["typeID"], d["workerID"]
        self.timeStamp, self.data, self.kind = d["timeStamp"], dict(d["data"]), d.get("kind", "meta")
        return self

    def __eq__(self, other):
        return isinstance(other, StorageMetaData) and self.to_dict() == other.to_dict()

    def __hash__(self):
        return hash((self.sessionID, self.typeID, self.workerID, self.timeStamp))


class SbeStorageMetaData(StorageMetaData):
    """The reference's constructor order: (timeStamp, sessionID, typeID, workerID, initType, updateType[, extra])."""

    def __init__(self, timeStamp=0, sessionID=None, typeID=None, workerID=None, initTypeClass=None,
                 updateTypeClass=None, extraMeta=None):
        super().__init__(sessionID, typeID, workerID, initTypeClass, updateTypeClass, timeStamp, extraMeta)


class StatsStorageEvent:
    NewSessionID, NewTypeID, NewWorkerID, PostMetaData, PostStaticInfo, PostUpdate = (
        "NewSessionID", "NewTypeID", "NewWorkerID", "PostMetaData", "PostStaticInfo", "PostUpdate")

    def __init__(self, storage, eventType, sessionID, typeID, workerID, timestamp):
        self.statsStorage, self.eventType = storage, eventType
        self.sessionID, self.typeID, self.workerID, self.timestamp = sessionID, typeID, workerID, timestamp


class StatsStorageListener:
    def notify(self, event):
        pass


class StatsStorageRouter:
    def putStorageMetaData(self, meta):
        raise NotImplementedError

    def putStaticInfo(self, rec):
        raise NotImplementedError

    def putUpdate(self, rec):
        raise NotImplementedError


class CollectionStatsStorageRouter(StatsStorageRouter):
    def __init__(self, metaStorage=None, staticInfoStorage=None, updateStorage=None):
        self.meta = [] if metaStorage is None else metaStorage
        self.static = [] if staticInfoStorage is None else staticInfoStorage
        self.updates = [] if updateStorage is None else updateStorage

    def putStorageMetaData(self, m):
        self.meta.extend(m if isinstance(m, (list, tuple)) else [m])

    def putStaticInfo(self, r):
        self.static.extend(r if isinstance(r, (list, tuple)) else [r])

    def putUpdate(self, r):
        self.updates.extend(r if isinstance(r, (list, tuple)) else [r])


class BaseCollectionStatsStorage(StatsStorageRouter):
    """Storage queries on top of three record maps (meta, static, updates) — shared by the in-memory and SQLite
    stores; the SQLite store overrides persistence."""

    def __init__(self):
        self._lock = threading.RLock()
        self.listeners = []
        self.closed = False

    # --- events
    def registerStatsStorageListener(self, l):
        self.listeners.append(l)

    def deregisterStatsStorageListener(self, l):
        self.listeners = [x for x in self.listeners if x is not l]

    def removeAllListeners(self):
        self.listeners = []

    def getListeners(self):
        return list(self.listeners)

    def _notify(self, kind, r, new_session, new_type, new_worker):
        evs = []
        if new_session:
            evs.append(StatsStorageEvent.NewSessionID)
        if new_type:
            evs.append(StatsStorageEvent.NewTypeID)
        if new_worker:
            evs.append(StatsStorageEvent.NewWorkerID)
        evs.append(kind)
        for l in self.listeners:
            for e in evs:
                l.notify(StatsStorageEvent(self, e, r.sessionID, r.typeID, r.workerID, r.timeStamp))

    def isClosed(self):
        return self.closed

    def close(self):
        self.closed = True


class InMemoryStatsStorage(BaseCollectionStatsStorage):
    def __init__(self):
        super().__init__()
        self.meta = {}          # (session, type) -> StorageMetaData
        self.static = {}        # (session, type, worker) -> Persistable
        self.updates = {}       # (session, type, worker) -> {timestamp: Persistable}

    def _ids(self):
        s = {k[0] for k in self.static} | {k[0] for k in self.updates} | {k[0] for k in self.meta}
        return s

    def _put(self, kind, r):
        with self._lock:
            new_s = r.sessionID not in self._ids()
            new_t = not any(k[0] == r.sessionID and k[1] == r.typeID for k in list(self.static) + list(self.updates))
            new_w = not any(k == (r.sessionID, r.typeID, r.workerID) for k in list(self.static) + list(self.updates))
            if kind == StatsStorageEvent.PostMetaData:
                self.meta[(r.sessionID, r.typeID)] = r
            elif kind == StatsStorageEvent.PostStaticInfo:
                self.static[(r.sessionID, r.typeID, r.workerID)] = r
            else:
                self.updates.setdefault((r.sessionID, r.typeID, r.workerID), {})[r.timeStamp] = r
        self._notify(kind, r, new_s, new_t, new_w)

    def putStorageMetaData(self, m):
        for x in (m if isinstance(m, (list, tuple)) else [m]):
            self._put(StatsStorageEvent.PostMetaData, x)

    def putStaticInfo(self, r):
        for x in (r if isinstance(r, (list, tuple)) else [r]):
            self._put(StatsStorageEvent.PostStaticInfo, x)

    def putUpdate(self, r):
        for x in (r if isinstance(r, (list, tuple)) else [r]):
            self._put(StatsStorageEvent.PostUpdate, x)

    # --- queries (StatsStorage API)
    def listSessionIDs(self):
        return sorted(self._ids())

    def sessionExists(self, s):
        return s in self._ids()

    def getStaticInfo(self, s, t, w):
        return self.static.get((s, t, w))

    def getAllStaticInfos(self, s, t):
        return [v for k, v in sorted(self.static.items()) if k[0] == s and k[1] == t]

    def listTypeIDsForSession(self, s):
        return sorted({k[1] for k in list(self.static) + list(self.updates) if k[0] == s})

    def listWorkerIDsForSession(self, s):
        return sorted({k[2] for k in list(self.static) + list(self.updates) if k[0] == s})

    def listWorkerIDsForSessionAndType(self, s, t):
        return sorted({k[2] for k in list(self.static) + list(self.updates) if k[0] == s and k[1] == t})

    def getNumUpdateRecordsFor(self, s, t=None, w=None):
        return sum(len(v) for k, v in self.updates.items()
                   if k[0] == s and (t is None or k[1] == t) and (w is None or k[2] == w))

    def _series(self, s, t, w):
        return self.updates.get((s, t, w), {})

    def getLatestUpdate(self, s, t, w):
        d = self._series(s, t, w)
        return d[max(d)] if d else None

    def getUpdate(self, s, t, w, ts):
        return self._series(s, t, w).get(ts)

    def getLatestUpdateAllWorkers(self, s, t):
        return [self.getLatestUpdate(s, t, w) for w in self.listWorkerIDsForSessionAndType(s, t)
                if self.getLatestUpdate(s, t, w) is not None]

    def getAllUpdatesAfter(self, s, t, w_or_ts, ts=None):
        if ts is None:
            out = []
            for w in self.listWorkerIDsForSessionAndType(s, t):
                out.extend(self.getAllUpdatesAfter(s, t, w, w_or_ts))
            return sorted(out, key=lambda r: r.timeStamp)
        d = self._series(s, t, w_or_ts)
        return [d[k] for k in sorted(d) if k > ts]

    def getAllUpdateTimes(self, s, t, w):
        return sorted(self._series(s, t, w))

    def getUpdates(self, s, t, w, timestamps):
        d = self._series(s, t, w)
        return [d[x] for x in timestamps if x in d]

    def getStorageMetaData(self, s, t):
        return self.meta.get((s, t))


class FileStatsStorage(InMemoryStatsStorage):
    """SQLite-backed persistent store (J7FileStatsStorage): every record is written through to the file, and an
    existing file is loaded on open, so a UI can be pointed at a finished run's stats file."""

    def __init__(self, path):
        super().__init__()
        self.path = path
        self.db = sqlite3.connect(path, check_same_thread=False)
        self.db.execute("create table if not exists records (kind text, session text, type text, worker text, "
                        "ts integer, payload blob)")
        self.db.commit()
        for kind, payload in self.db.execute("select kind, payload from records order by rowid"):
            r = Persistable.decode(payload)
            if kind == StatsStorageEvent.PostMetaData:
                self.meta[(r.sessionID, r.typeID)] = r
            elif kind == StatsStorageEvent.PostStaticInfo:
                self.static[(r.sessionID, r.typeID, r.workerID)] = r
            else:
                self.updates.setdefault((r.sessionID, r.typeID, r.workerID), {})[r.timeStamp] = r

    def _put(self, kind, r):
        with self._lock:
            self.db.execute("insert into records values (?,?,?,?,?,?)",
                            (kind, r.sessionID, r.typeID, r.workerID, r.timeStamp, r.encode()))
            self.db.commit()
        super()._put(kind, r)

    def close(self):
        super().close()
        self.db.close()


J7FileStatsStorage = FileStatsStorage
MapDBStatsStorage = FileStatsStorage


class RemoteUIStatsStorageRouter(StatsStorageRouter):
    """POSTs records to a remote UIServer's /remoteReceive endpoint (RemoteUIStatsStorageRouter.java), with a
    bounded retry queue so training never blocks on the UI."""

    def __init__(self, address, maxRetryCount=10, retryBackoffSeconds=1.0):
        self.url = address.rstrip("/") + "/remoteReceive"
        self.maxRetry, self.backoff = maxRetryCount, retryBackoffSeconds
        self.failures = 0

    def _post(self, kind, r):
        body = json.dumps({"type": kind, "record": r.to_dict()}).encode()
        for attempt in range(self.maxRetry):
            try:
                req = urllib.request.Request(self.url, body, {"Content-Type": "application/json"})
                with urllib.request.urlopen(req, timeout=10) as resp:
                    resp.read()
                return True
            except OSError:
                self.failures += 1
                time.sleep(self.backoff * (attempt + 1) * 0.1)
        return False

    def putStorageMetaData(self, m):
        for x in (m if isinstance(m, (list, tuple)) else [m]):
            self._post("meta", x)

    def putStaticInfo(self, r):
        for x in (r if isinstance(r, (list, tuple)) else [r]):
            self._post("static", x)

    def putUpdate(self, r):
        for x in (r if isinstance(r, (list, tuple)) else [r]):
            self._post("update", x)
