"""UIDProvider: a per-process id and a per-machine id for stats / UI sessions and worker names (reference
deeplearning4j-core/src/main/java/org/deeplearning4j/util/UIDProvider.java). The process id is a random UUID drawn
once per process (the reference's "JVM UID"); the hardware id hashes the host name and the primary MAC address."""
import hashlib
import socket
import uuid

_PROCESS_UID = uuid.uuid4().hex


class UIDProvider:
    @staticmethod
    def getJVMUID():
        return _PROCESS_UID

    getProcessUID = getJVMUID

    @staticmethod
    def getHardwareUID():
        key = f"{socket.gethostname()}|{uuid.getnode():012x}"
        return hashlib.sha1(key.encode()).hexdigest()[:16]
