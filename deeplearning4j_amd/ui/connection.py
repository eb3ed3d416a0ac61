"""Where a remote UI lives (reference deeplearning4j-core/src/main/java/org/deeplearning4j/ui/UiConnectionInfo.java):
scheme / address / port / path, with paths normalised to "/a/b/" (duplicate slashes collapsed). Used by the
remote stats router to build its POST URL."""
import re


def _norm(*parts):
    segs = [p for part in parts if part for p in re.split(r"/+", part) if p]
    return "/" + "".join(s + "/" for s in segs) if segs else "/"


class UiConnectionInfo:
    def __init__(self, address="localhost", port=9000, path="", useHttps=False, login=None, password=None):
        self.address, self.port, self.path, self.useHttps = address, int(port), path, bool(useHttps)
        self.login, self.password = login, password
        self.sessionId = None

    def getFirstPart(self):
        return f"{'https' if self.useHttps else 'http'}://{self.address}:{self.port}"

    def getSecondPart(self, nPath=None):
        return _norm(self.path, nPath)

    def getFullAddress(self, nPath=None):
        return self.getFirstPart() + self.getSecondPart(nPath)

    def setSessionId(self, sid):
        self.sessionId = sid

    def getSessionId(self):
        return self.sessionId

    class Builder:
        def __init__(self):
            self._kw = {}

        def setAddress(self, a):
            self._kw["address"] = a
            return self

        def setPort(self, p):
            self._kw["port"] = int(p)
            return self

        def setPath(self, p):
            self._kw["path"] = p
            return self

        def enableHttps(self, b):
            self._kw["useHttps"] = bool(b)
            return self

        def setLogin(self, login):
            self._kw["login"] = login
            return self

        def setPassword(self, pw):
            self._kw["password"] = pw
            return self

        def build(self):
            return UiConnectionInfo(**self._kw)
