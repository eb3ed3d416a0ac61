"""Dependency-free AWS API client: Signature Version 4 request signing plus the two wire protocols the provisioning
classes need — the EC2 Query protocol (form-encoded request, XML response) and the EMR JSON 1.1 protocol
(``X-Amz-Target`` header, JSON body). The reference reaches these services through the AWS Java SDK
(aws/ec2/Ec2BoxCreator.java:79-215, aws/emr/SparkEMRClient.java:58-250); this image has neither boto3 nor network,
so the client is plain ``urllib`` over a configurable endpoint (tests point it at a local fake service that checks
the signature).

Only stdlib: ``hashlib`` / ``hmac`` for SigV4, ``urllib.request`` for transport, ``xml.etree`` for EC2 responses.
"""
import datetime
import hashlib
import hmac
import json
import os
import urllib.parse
import urllib.request
import xml.etree.ElementTree as ET


class AwsError(RuntimeError):
    def __init__(self, status, code, message):
        super().__init__(f"AWS {status} {code}: {message}")
        self.status, self.code, self.message = status, code, message


def _sha256(b):
    return hashlib.sha256(b).hexdigest()


def _hmac(key, msg):
    return hmac.new(key, msg.encode("utf-8"), hashlib.sha256).digest()


def _uri_encode(s, safe="-_.~"):
    return urllib.parse.quote(s, safe=safe)


class Credentials:
    """Access key / secret / optional session token; defaults from the standard AWS environment variables."""

    def __init__(self, accessKey=None, secretKey=None, sessionToken=None):
        self.accessKey = accessKey or os.environ.get("AWS_ACCESS_KEY_ID") or os.environ.get("AWS_ACCESS_KEY")
        self.secretKey = secretKey or os.environ.get("AWS_SECRET_ACCESS_KEY") or os.environ.get("AWS_SECRET_KEY")
        self.sessionToken = sessionToken or os.environ.get("AWS_SESSION_TOKEN")
        if not self.accessKey or not self.secretKey:
            raise ValueError("AWS credentials missing: pass accessKey/secretKey or set AWS_ACCESS_KEY_ID / "
                             "AWS_SECRET_ACCESS_KEY")


def canonical_request(method, path, query, headers, payload_hash):
    """SigV4 canonical request: method, URI-encoded path, sorted query, lower-cased sorted headers with trimmed
    values, the signed-header list and the payload hash. Returns (canonical_request, signed_headers)."""
    q = sorted((_uri_encode(k), _uri_encode(v)) for k, v in query)
    cq = "&".join(f"{k}={v}" for k, v in q)
    hs = sorted((k.lower(), " ".join(str(v).strip().split())) for k, v in headers.items())
    ch = "".join(f"{k}:{v}\n" for k, v in hs)
    signed = ";".join(k for k, _ in hs)
    cpath = _uri_encode(path or "/", safe="-_.~/")
    return "\n".join([method, cpath, cq, ch, signed, payload_hash]), signed


def sign(method, url, headers, body, creds, region, service, now=None):
    """Add ``X-Amz-Date`` (and the session token) and the SigV4 ``Authorization`` header to ``headers``; returns
    the dict of headers to send. ``now`` (a UTC datetime) pins the timestamp for tests."""
    now = now or datetime.datetime.now(datetime.timezone.utc)
    amz_date = now.strftime("%Y%m%dT%H%M%SZ")
    day = amz_date[:8]
    u = urllib.parse.urlsplit(url)
    h = dict(headers)
    h.setdefault("Host", u.netloc)
    h["X-Amz-Date"] = amz_date
    if creds.sessionToken:
        h["X-Amz-Security-Token"] = creds.sessionToken
    payload_hash = _sha256(body or b"")
    creq, signed = canonical_request(method, u.path, urllib.parse.parse_qsl(u.query, keep_blank_values=True), h,
                                     payload_hash)
    scope = f"{day}/{region}/{service}/aws4_request"
    sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, _sha256(creq.encode("utf-8"))])
    k = _hmac(("AWS4" + creds.secretKey).encode("utf-8"), day)
    k = _hmac(k, region)
    k = _hmac(k, service)
    k = _hmac(k, "aws4_request")
    sig = hmac.new(k, sts.encode("utf-8"), hashlib.sha256).hexdigest()
    h["Authorization"] = (f"AWS4-HMAC-SHA256 Credential={creds.accessKey}/{scope}, SignedHeaders={signed}, "
                          f"Signature={sig}")
    return h


class _Client:
    def __init__(self, service, region="us-east-1", endpoint=None, credentials=None, timeout=60.0):
        self.service, self.region = service, region
        self.endpoint = (endpoint or os.environ.get(f"DL4J_AMD_{service.upper()}_ENDPOINT")
                         or f"https://{service if service != 'elasticmapreduce' else 'elasticmapreduce'}."
                            f"{region}.amazonaws.com").rstrip("/")
        self.creds = credentials or Credentials()
        self.timeout = timeout

    def _send(self, method, headers, body):
        url = self.endpoint + "/"
        h = sign(method, url, headers, body, self.creds, self.region, self.service)
        req = urllib.request.Request(url, data=body, headers=h, method=method)
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                return r.status, r.read()
        except urllib.error.HTTPError as e:
            return e.code, e.read()


def _strip_ns(elem):
    for e in elem.iter():
        if "}" in e.tag:
            e.tag = e.tag.split("}", 1)[1]
    return elem


def flatten_query(params, prefix=""):
    """EC2 Query serialisation of nested params: lists become ``Name.1``, ``Name.2``, dicts ``Name.Key``."""
    out = []
    for k, v in params.items():
        name = f"{prefix}{k}"
        if isinstance(v, dict):
            out += flatten_query(v, name + ".")
        elif isinstance(v, (list, tuple)):
            for i, item in enumerate(v, 1):
                if isinstance(item, dict):
                    out += flatten_query(item, f"{name}.{i}.")
                else:
                    out.append((f"{name}.{i}", str(item)))
        elif isinstance(v, bool):
            out.append((name, "true" if v else "false"))
        elif v is not None:
            out.append((name, str(v)))
    return out


class Ec2Client(_Client):
    """EC2 Query API (API version 2016-11-15): POST form body, XML response (namespace stripped)."""
    VERSION = "2016-11-15"

    def __init__(self, region="us-east-1", endpoint=None, credentials=None, timeout=60.0):
        super().__init__("ec2", region, endpoint, credentials, timeout)

    def call(self, action, **params):
        form = [("Action", action), ("Version", self.VERSION)] + flatten_query(params)
        body = urllib.parse.urlencode(form).encode("utf-8")
        status, data = self._send("POST", {"Content-Type": "application/x-www-form-urlencoded; charset=utf-8"},
                                  body)
        root = _strip_ns(ET.fromstring(data))
        if status >= 300 or root.tag == "Response" and root.find(".//Errors") is not None:
            err = root.find(".//Error")
            code = err.findtext("Code") if err is not None else str(status)
            msg = err.findtext("Message") if err is not None else data.decode("utf-8", "replace")
            raise AwsError(status, code, msg)
        return root

    @staticmethod
    def instances(root):
        """[{id, state, publicDns, privateIp, type}] from a RunInstances / DescribeInstances response."""
        out = []
        for it in root.iter("item"):
            iid = it.findtext("instanceId")
            if iid is None or it.find("instanceState") is None and it.find("currentState") is None:
                continue
            st = it.find("instanceState") if it.find("instanceState") is not None else it.find("currentState")
            out.append({"id": iid, "state": st.findtext("name"), "publicDns": it.findtext("dnsName") or "",
                        "privateIp": it.findtext("privateIpAddress") or "", "type": it.findtext("instanceType")})
        return out


class EmrClient(_Client):
    """EMR JSON 1.1 API: ``X-Amz-Target: ElasticMapReduce.<Action>``, JSON in and out."""

    def __init__(self, region="us-east-1", endpoint=None, credentials=None, timeout=60.0):
        super().__init__("elasticmapreduce", region, endpoint, credentials, timeout)

    def call(self, action, **params):
        body = json.dumps(params).encode("utf-8")
        status, data = self._send("POST", {"Content-Type": "application/x-amz-json-1.1",
                                           "X-Amz-Target": f"ElasticMapReduce.{action}"}, body)
        doc = json.loads(data.decode("utf-8") or "{}")
        if status >= 300:
            raise AwsError(status, doc.get("__type", str(status)), doc.get("message") or doc.get("Message", ""))
        return doc
