"""Kafka wire-protocol client (and a small protocol-level broker for tests) behind the streaming ``Broker`` interface,
so ``NDArrayPublisher`` / ``NDArrayConsumer`` / ``NDArrayPubSubRoute`` / ``DL4jServeRouteBuilder`` can run over a real
Kafka cluster (reference dl4j-streaming: Camel kafka: endpoints, STRM:kafka/NDArrayPublisher.java,
NDArrayConsumer.java, routes/DL4jServeRouteBuilder.java:48-92).

No Kafka client library is in this image, so the protocol is spoken directly over TCP:
  * request header v1 (api_key, api_version, correlation_id, client_id), size-prefixed frames;
  * Metadata v1 (partition leaders), Produce v3, Fetch v4, ListOffsets v1 — the versions every broker from 0.11
    through 4.x accepts — with RecordBatch v2 record sets (magic 2, CRC-32C over attributes..records, zig-zag
    varint record fields).
``KafkaBroker`` implements ``subscribe`` / ``unsubscribe`` / ``publish``: a subscription starts at the partition's
latest offset (the in-process broker's "messages published after subscribing") and a fetch thread long-polls into
the subscriber's queue. ``MiniKafkaServer`` implements the same four APIs over an in-memory log for the tests.
"""
import socket
import socketserver
import struct
import threading
import time
import queue

__all__ = ["KafkaBroker", "MiniKafkaServer", "crc32c", "encode_record_batch", "decode_record_batches"]

API_PRODUCE, API_FETCH, API_LIST_OFFSETS, API_METADATA = 0, 1, 2, 3
V_PRODUCE, V_FETCH, V_LIST_OFFSETS, V_METADATA = 3, 4, 1, 1
ERR_NONE, ERR_UNKNOWN_TOPIC, ERR_OFFSET_OUT_OF_RANGE = 0, 3, 1

# --------------------------------------------------------------------------------------------- CRC-32C (Castagnoli)
_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)


def crc32c(data, crc=0):
    crc ^= 0xFFFFFFFF
    tab = _CRC_TABLE
    for b in data:
        crc = tab[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


# --------------------------------------------------------------------------------------------- primitive codecs
class _W:
    def __init__(self):
        self.parts = []

    def i8(self, v):
        self.parts.append(struct.pack(">b", v)); return self

    def i16(self, v):
        self.parts.append(struct.pack(">h", v)); return self

    def i32(self, v):
        self.parts.append(struct.pack(">i", v)); return self

    def i64(self, v):
        self.parts.append(struct.pack(">q", v)); return self

    def u32(self, v):
        self.parts.append(struct.pack(">I", v)); return self

    def string(self, s):
        if s is None:
            return self.i16(-1)
        b = s.encode("utf-8")
        self.i16(len(b)); self.parts.append(b); return self

    def bytes_(self, b):
        if b is None:
            return self.i32(-1)
        self.i32(len(b)); self.parts.append(bytes(b)); return self

    def raw(self, b):
        self.parts.append(bytes(b)); return self

    def varint(self, v):
        z = (v << 1) ^ (v >> 63)                     # zig-zag
        out = bytearray()
        while True:
            if z & ~0x7F:
                out.append((z & 0x7F) | 0x80)
                z >>= 7
            else:
                out.append(z)
                break
        self.parts.append(bytes(out)); return self

    def array(self, items, fn):
        if items is None:
            return self.i32(-1)
        self.i32(len(items))
        for it in items:
            fn(self, it)
        return self

    def getvalue(self):
        return b"".join(self.parts)


class _R:
    def __init__(self, buf, pos=0):
        self.b, self.p = memoryview(buf), pos

    def _u(self, fmt, n):
        v = struct.unpack_from(fmt, self.b, self.p)[0]
        self.p += n
        return v

    def i8(self):
        return self._u(">b", 1)

    def i16(self):
        return self._u(">h", 2)

    def i32(self):
        return self._u(">i", 4)

    def i64(self):
        return self._u(">q", 8)

    def u32(self):
        return self._u(">I", 4)

    def string(self):
        n = self.i16()
        if n < 0:
            return None
        s = bytes(self.b[self.p:self.p + n]).decode("utf-8")
        self.p += n
        return s

    def bytes_(self):
        n = self.i32()
        if n < 0:
            return None
        s = bytes(self.b[self.p:self.p + n])
        self.p += n
        return s

    def varint(self):
        shift = z = 0
        while True:
            c = self.b[self.p]
            self.p += 1
            z |= (c & 0x7F) << shift
            if not c & 0x80:
                break
            shift += 7
        return (z >> 1) ^ -(z & 1)

    def array(self, fn):
        n = self.i32()
        return None if n < 0 else [fn(self) for _ in range(n)]

    def remaining(self):
        return len(self.b) - self.p


# --------------------------------------------------------------------------------------------- record batches
def encode_record_batch(records, base_offset=0, base_timestamp=None):
    """RecordBatch v2 of ``records`` = [(key bytes|None, value bytes|None), ...]."""
    ts = int(time.time() * 1000) if base_timestamp is None else base_timestamp
    body = _W()
    for i, (k, v) in enumerate(records):
        r = _W().i8(0).varint(0).varint(i)
        if k is None:
            r.varint(-1)
        else:
            r.varint(len(k)).raw(k)
        if v is None:
            r.varint(-1)
        else:
            r.varint(len(v)).raw(v)
        r.varint(0)                                   # no headers
        rb = r.getvalue()
        body.varint(len(rb)).raw(rb)
    tail = (_W().i16(0).i32(len(records) - 1).i64(ts).i64(ts).i64(-1).i16(-1).i32(-1).i32(len(records))
            .raw(body.getvalue()).getvalue())
    crc = crc32c(tail)
    after_len = _W().i32(0).i8(2).u32(crc).raw(tail).getvalue()    # partitionLeaderEpoch, magic, crc, ...
    return _W().i64(base_offset).i32(len(after_len)).raw(after_len).getvalue()


def decode_record_batches(buf, verify=True):
    """[(offset, key, value), ...] of every complete RecordBatch v2 in ``buf`` (a trailing partial batch, which a
    fetch may return, is ignored)."""
    out = []
    r = _R(buf)
    while r.remaining() >= 12:
        base = r.i64()
        blen = r.i32()
        if r.remaining() < blen:
            break
        end = r.p + blen
        r.i32()                                       # partition leader epoch
        magic = r.i8()
        if magic != 2:
            raise ValueError(f"unsupported record batch magic {magic}")
        crc = r.u32()
        if verify and crc32c(bytes(r.b[r.p:end])) != crc:
            raise ValueError("record batch CRC-32C mismatch")
        r.i16(); r.i32(); r.i64(); r.i64(); r.i64(); r.i16(); r.i32()
        n = r.i32()
        for _ in range(n):
            r.varint()                                # record length
            r.i8(); r.varint()
            off = r.varint()
            kl = r.varint()
            k = None if kl < 0 else bytes(r.b[r.p:r.p + kl])
            r.p += max(kl, 0)
            vl = r.varint()
            v = None if vl < 0 else bytes(r.b[r.p:r.p + vl])
            r.p += max(vl, 0)
            for _ in range(r.varint()):               # headers
                hk = r.varint(); r.p += hk
                hv = r.varint(); r.p += max(hv, 0)
            out.append((base + off, k, v))
        r.p = end
    return out


# --------------------------------------------------------------------------------------------- client
class _Conn:
    def __init__(self, host, port, client_id, timeout):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.client_id = client_id
        self.corr = 0
        self.lock = threading.Lock()

    def request(self, api, ver, body):
        with self.lock:
            self.corr += 1
            hdr = _W().i16(api).i16(ver).i32(self.corr).string(self.client_id).getvalue()
            msg = hdr + body
            self.sock.sendall(struct.pack(">i", len(msg)) + msg)
            n = struct.unpack(">i", self._read(4))[0]
            data = self._read(n)
        r = _R(data)
        if r.i32() != self.corr:
            raise IOError("Kafka response correlation id mismatch")
        return r

    def _read(self, n):
        buf = bytearray()
        while len(buf) < n:
            chunk = self.sock.recv(n - len(buf))
            if not chunk:
                raise IOError("Kafka connection closed")
            buf += chunk
        return bytes(buf)

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass


class KafkaError(IOError):
    pass


class KafkaBroker:
    """The streaming ``Broker`` interface over Kafka. ``bootstrap`` = "host:port[,host:port...]". Messages are the
    record values (str -> UTF-8); a subscription reads partition ``partition`` from its latest offset."""

    def __init__(self, bootstrap, client_id="dl4j-amd", partition=0, timeout=10.0, max_wait_ms=100):
        self.bootstrap = [(h, int(p)) for h, p in (x.rsplit(":", 1) for x in bootstrap.split(","))]
        self.client_id, self.partition, self.timeout, self.max_wait = client_id, partition, timeout, max_wait_ms
        self._conns = {}
        self._leaders = {}
        self._nodes = {}
        self._subs = {}
        self._lock = threading.Lock()

    # ---- connections / metadata
    def _conn(self, addr):
        with self._lock:
            c = self._conns.get(addr)
            if c is None:
                c = self._conns[addr] = _Conn(addr[0], addr[1], self.client_id, self.timeout)
            return c

    def metadata(self, topics=None):
        body = _W().array(topics, lambda w, t: w.string(t)).getvalue()
        r = self._conn(self.bootstrap[0]).request(API_METADATA, V_METADATA, body)
        brokers = r.array(lambda r: (r.i32(), r.string(), r.i32(), r.string()))
        r.i32()                                       # controller id
        topics_md = r.array(lambda r: (r.i16(), r.string(), r.i8(),
                                       r.array(lambda r: (r.i16(), r.i32(), r.i32(),
                                                          r.array(lambda r: r.i32()),
                                                          r.array(lambda r: r.i32())))))
        self._nodes = {nid: (host, port) for nid, host, port, _ in brokers}
        out = {}
        for err, name, _internal, parts in topics_md:
            out[name] = (err, {p: leader for _e, p, leader, _r, _i in parts})
            for p, leader in out[name][1].items():
                self._leaders[(name, p)] = leader
        return out

    def _leader(self, topic, partition):
        key = (topic, partition)
        if key not in self._leaders:
            md = self.metadata([topic])
            err = md.get(topic, (ERR_UNKNOWN_TOPIC, {}))[0]
            if key not in self._leaders:
                raise KafkaError(f"no leader for {topic}[{partition}] (error {err})")
        return self._conn(self._nodes[self._leaders[key]])

    # ---- produce / fetch / offsets
    def produce(self, topic, values, partition=None, acks=1):
        partition = self.partition if partition is None else partition
        recs = [(None, v.encode("utf-8") if isinstance(v, str) else bytes(v)) for v in values]
        batch = encode_record_batch(recs)
        body = (_W().string(None).i16(acks).i32(int(self.timeout * 1000))
                .array([topic], lambda w, t: w.string(t).array([partition], lambda w, p: w.i32(p).bytes_(batch)))
                .getvalue())
        r = self._leader(topic, partition).request(API_PRODUCE, V_PRODUCE, body)
        resp = r.array(lambda r: (r.string(), r.array(lambda r: (r.i32(), r.i16(), r.i64(), r.i64()))))
        for _t, parts in resp:
            for _p, err, base, _ts in parts:
                if err != ERR_NONE:
                    raise KafkaError(f"produce to {topic}[{partition}] failed: error {err}")
                return base

    def list_offset(self, topic, partition=None, latest=True):
        partition = self.partition if partition is None else partition
        body = (_W().i32(-1).array([topic], lambda w, t: w.string(t).array(
            [partition], lambda w, p: w.i32(p).i64(-1 if latest else -2))).getvalue())
        r = self._leader(topic, partition).request(API_LIST_OFFSETS, V_LIST_OFFSETS, body)
        resp = r.array(lambda r: (r.string(), r.array(lambda r: (r.i32(), r.i16(), r.i64(), r.i64()))))
        _p, err, _ts, off = resp[0][1][0]
        if err != ERR_NONE:
            raise KafkaError(f"list offsets {topic}[{partition}]: error {err}")
        return off

    def fetch(self, topic, offset, partition=None, max_bytes=4 << 20, max_wait_ms=None, conn=None):
        """[(offset, key, value)] from ``offset`` on, and the high watermark. ``conn``: a dedicated connection to the
        partition leader (subscriptions long-poll on their own socket, so they never hold up produce requests)."""
        partition = self.partition if partition is None else partition
        mw = self.max_wait if max_wait_ms is None else max_wait_ms
        body = (_W().i32(-1).i32(mw).i32(1).i32(max_bytes).i8(0)
                .array([topic], lambda w, t: w.string(t).array(
                    [partition], lambda w, p: w.i32(p).i64(offset).i32(max_bytes))).getvalue())
        r = (conn or self._leader(topic, partition)).request(API_FETCH, V_FETCH, body)
        r.i32()                                       # throttle
        resp = r.array(lambda r: (r.string(), r.array(lambda r: (
            r.i32(), r.i16(), r.i64(), r.i64(), r.array(lambda r: (r.i64(), r.i64())), r.bytes_()))))
        _p, err, hw, _lso, _ab, records = resp[0][1][0]
        if err != ERR_NONE:
            raise KafkaError(f"fetch {topic}[{partition}] at {offset}: error {err}")
        recs = [x for x in decode_record_batches(records or b"") if x[0] >= offset]
        return recs, hw

    # ---- Broker interface
    def publish(self, topic, message):
        self.produce(topic, [message])
        return 1

    def subscribe(self, topic, maxsize=0):
        q = queue.Queue(maxsize)
        stop = threading.Event()
        start = self.list_offset(topic)

        self._leader(topic, self.partition)
        addr = self._nodes[self._leaders[(topic, self.partition)]]
        conn = _Conn(addr[0], addr[1], self.client_id, self.timeout)

        def run():
            off = start
            while not stop.is_set():
                try:
                    recs, _hw = self.fetch(topic, off, conn=conn)
                except (KafkaError, OSError):
                    if stop.is_set():
                        break
                    time.sleep(0.05)
                    continue
                for o, _k, v in recs:
                    q.put(v.decode("utf-8") if v is not None else None)
                    off = o + 1
            conn.close()
        t = threading.Thread(target=run, daemon=True, name=f"kafka-fetch-{topic}")
        with self._lock:
            self._subs[id(q)] = (stop, t)
        t.start()
        return q

    def unsubscribe(self, topic, q):
        with self._lock:
            s = self._subs.pop(id(q), None)
        if s is not None:
            s[0].set()
            s[1].join(timeout=2.0)

    def close(self):
        for key in list(self._subs):
            stop, t = self._subs.pop(key)
            stop.set()
            t.join(timeout=2.0)
        for c in self._conns.values():
            c.close()
        self._conns.clear()


# --------------------------------------------------------------------------------------------- test broker
class MiniKafkaServer:
    """A single-node, in-memory Kafka-protocol server (Metadata v1, Produce v3, Fetch v4, ListOffsets v1) for tests
    and local pipelines. Topics are auto-created with one partition; each produced batch is stored as the batch bytes
    re-based to its log offset, and a fetch returns whole batches from the one holding the fetch offset."""

    def __init__(self, host="127.0.0.1", port=0, node_id=1):
        self.logs = {}                                 # (topic, partition) -> [(base_offset, n, batch_bytes)]
        self.cond = threading.Condition()
        self.node_id = node_id
        server = self

        class Handler(socketserver.BaseRequestHandler):
            def handle(self):
                sock = self.request
                while True:
                    hdr = _recv_exact(sock, 4)
                    if hdr is None:
                        return
                    data = _recv_exact(sock, struct.unpack(">i", hdr)[0])
                    if data is None:
                        return
                    resp = server._dispatch(data)
                    sock.sendall(struct.pack(">i", len(resp)) + resp)

        class TCP(socketserver.ThreadingMixIn, socketserver.TCPServer):
            daemon_threads = True
            allow_reuse_address = True

        self._srv = TCP((host, port), Handler)
        self.host, self.port = self._srv.server_address
        self._t = threading.Thread(target=self._srv.serve_forever, daemon=True, name="mini-kafka")

    @property
    def bootstrap(self):
        return f"{self.host}:{self.port}"

    def start(self):
        self._t.start()
        return self

    def stop(self):
        self._srv.shutdown()
        self._srv.server_close()

    def _log(self, topic, p):
        return self.logs.setdefault((topic, p), [])

    def _end(self, log):
        return log[-1][0] + log[-1][1] if log else 0

    def _dispatch(self, data):
        r = _R(data)
        api, ver, corr = r.i16(), r.i16(), r.i32()
        r.string()
        w = _W().i32(corr)
        if api == API_METADATA and ver == V_METADATA:
            topics = r.array(lambda r: r.string())
            with self.cond:
                names = topics if topics is not None else sorted({t for t, _ in self.logs})
                for t in names:
                    self._log(t, 0)
            w.array([(self.node_id, self.host, self.port)], lambda w, b: w.i32(b[0]).string(b[1]).i32(b[2]).string(None))
            w.i32(self.node_id)
            w.array(names, lambda w, t: w.i16(0).string(t).i8(0).array(
                [0], lambda w, p: w.i16(0).i32(p).i32(self.node_id).array([self.node_id], lambda w, x: w.i32(x))
                .array([self.node_id], lambda w, x: w.i32(x))))
        elif api == API_PRODUCE and ver == V_PRODUCE:
            r.string(); r.i16(); r.i32()
            topics = r.array(lambda r: (r.string(), r.array(lambda r: (r.i32(), r.bytes_()))))
            res = []
            with self.cond:
                for t, parts in topics:
                    pr = []
                    for p, batch in parts:
                        log = self._log(t, p)
                        base = self._end(log)
                        try:
                            recs = decode_record_batches(batch)
                        except ValueError:
                            pr.append((p, 2, -1))     # CORRUPT_MESSAGE
                            continue
                        rebased = struct.pack(">q", base) + batch[8:]
                        log.append((base, len(recs), rebased))
                        pr.append((p, 0, base))
                    res.append((t, pr))
                self.cond.notify_all()
            w.array(res, lambda w, tr: w.string(tr[0]).array(
                tr[1], lambda w, x: w.i32(x[0]).i16(x[1]).i64(x[2]).i64(-1)))
            w.i32(0)
        elif api == API_LIST_OFFSETS and ver == V_LIST_OFFSETS:
            r.i32()
            topics = r.array(lambda r: (r.string(), r.array(lambda r: (r.i32(), r.i64()))))
            with self.cond:
                res = [(t, [(p, 0, -1, self._end(self._log(t, p)) if ts == -1 else 0) for p, ts in parts])
                       for t, parts in topics]
            w.array(res, lambda w, tr: w.string(tr[0]).array(
                tr[1], lambda w, x: w.i32(x[0]).i16(x[1]).i64(x[2]).i64(x[3])))
        elif api == API_FETCH and ver == V_FETCH:
            r.i32()
            max_wait = r.i32()
            r.i32(); r.i32(); r.i8()
            topics = r.array(lambda r: (r.string(), r.array(lambda r: (r.i32(), r.i64(), r.i32()))))
            deadline = time.time() + max_wait / 1000.0
            with self.cond:
                while time.time() < deadline and all(
                        self._end(self._log(t, p)) <= off for t, parts in topics for p, off, _ in parts):
                    self.cond.wait(max(0.0, deadline - time.time()))
                res = []
                for t, parts in topics:
                    pr = []
                    for p, off, maxb in parts:
                        log = self._log(t, p)
                        end = self._end(log)
                        if off > end:
                            pr.append((p, ERR_OFFSET_OUT_OF_RANGE, end, b""))
                            continue
                        out, size = [], 0
                        for base, n, b in log:
                            if base + n <= off:
                                continue
                            if out and size + len(b) > maxb:
                                break
                            out.append(b)
                            size += len(b)
                        pr.append((p, 0, end, b"".join(out)))
                    res.append((t, pr))
            w.i32(0)
            w.array(res, lambda w, tr: w.string(tr[0]).array(
                tr[1], lambda w, x: w.i32(x[0]).i16(x[1]).i64(x[2]).i64(x[2]).array([], None).bytes_(x[3])))
        else:
            raise IOError(f"MiniKafkaServer: unsupported api {api} v{ver}")
        return w.getvalue()


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        try:
            chunk = sock.recv(n - len(buf))
        except OSError:
            return None
        if not chunk:
            return None
        buf += chunk
    return bytes(buf)
