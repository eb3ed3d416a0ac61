"""SigV4 signing and the EC2 / EMR provisioning clients (aws/client.py, aws/__init__.py) against a local fake AWS
service that re-derives every request's signature (reference: aws/ec2/Ec2BoxCreator.java:58-215,
aws/emr/SparkEMRClient.java:58-250, aws/ec2/provision/HostProvisioner.java:53-270)."""
import datetime
import http.server
import json
import threading
import urllib.parse

import pytest

from deeplearning4j_amd import aws
from deeplearning4j_amd.aws import client as C

AK, SK = "AKIDEXAMPLE", "wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY"


def test_sigv4_matches_the_published_aws_example():
    """The IAM ListUsers example of the AWS SigV4 documentation (2015-08-30T12:36:00Z, us-east-1/iam)."""
    creds = C.Credentials(AK, SK)
    url = "https://iam.amazonaws.com/?Action=ListUsers&Version=2010-05-08"
    hdr = {"Content-Type": "application/x-www-form-urlencoded; charset=utf-8"}
    now = datetime.datetime(2015, 8, 30, 12, 36, 0, tzinfo=datetime.timezone.utc)
    creq, signed = C.canonical_request(
        "GET", "/", urllib.parse.parse_qsl("Action=ListUsers&Version=2010-05-08"),
        dict(hdr, Host="iam.amazonaws.com", **{"X-Amz-Date": "20150830T123600Z"}), C._sha256(b""))
    assert signed == "content-type;host;x-amz-date"
    assert C._sha256(creq.encode()) == "f536975d06c0309214f805bb90ccff089219ecd68b2577efef23edd43b7e1a59"
    h = C.sign("GET", url, hdr, b"", creds, "us-east-1", "iam", now=now)
    assert h["Authorization"].endswith(
        "Signature=5d672d79c15b13162d9279b0855cfba6789a8edb4c82c400e06b5924a6f2b5d7")
    assert "Credential=AKIDEXAMPLE/20150830/us-east-1/iam/aws4_request" in h["Authorization"]


def test_flatten_query_lists_and_dicts():
    q = C.flatten_query({"InstanceId": ["i-1", "i-2"], "LaunchSpecification": {"ImageId": "ami", "X": [1]},
                         "Flag": True, "Skip": None})
    assert q == [("InstanceId.1", "i-1"), ("InstanceId.2", "i-2"), ("LaunchSpecification.ImageId", "ami"),
                 ("LaunchSpecification.X.1", "1"), ("Flag", "true")]


class FakeAws:
    """EC2 Query + EMR JSON fake: verifies the SigV4 signature of every request, keeps instance / cluster state."""

    def __init__(self):
        self.calls, self.instances, self.clusters, self.steps = [], {}, {}, {}
        self.describe_count = 0
        fake = self

        class H(http.server.BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_POST(self):
                body = self.rfile.read(int(self.headers["Content-Length"]))
                fake.check_signature(self, body)
                target = self.headers.get("X-Amz-Target")
                if target:
                    code, out = fake.emr(target.split(".", 1)[1], json.loads(body))
                    data, ctype = json.dumps(out).encode(), "application/x-amz-json-1.1"
                else:
                    form = dict(urllib.parse.parse_qsl(body.decode()))
                    code, data, ctype = 200, fake.ec2(form).encode(), "text/xml"
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

        self.srv = http.server.HTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def check_signature(self, req, body):
        auth = req.headers["Authorization"]
        scope = auth.split("Credential=")[1].split(",")[0].split("/")
        signed = auth.split("SignedHeaders=")[1].split(",")[0].split(";")
        hdrs = {k: req.headers[k] for k in signed}
        creq, _ = C.canonical_request("POST", req.path.split("?")[0], [], hdrs, C._sha256(body))
        sts = "\n".join(["AWS4-HMAC-SHA256", req.headers["X-Amz-Date"], "/".join(scope[1:]),
                         C._sha256(creq.encode())])
        k = C._hmac(("AWS4" + SK).encode(), scope[1])
        for part in scope[2:]:
            k = C._hmac(k, part)
        import hashlib
        import hmac
        want = hmac.new(k, sts.encode(), hashlib.sha256).hexdigest()
        assert auth.endswith("Signature=" + want), "bad SigV4 signature"
        self.calls.append(req.headers.get("X-Amz-Target") or "ec2")

    def ec2(self, f):
        act = f["Action"]
        self.calls[-1] = act
        ids = [v for k, v in sorted(f.items()) if k.startswith("InstanceId.")]
        if act == "RunInstances":
            n = int(f["MaxCount"])
            new = [f"i-{len(self.instances) + j:04d}" for j in range(n)]
            for i in new:
                self.instances[i] = "pending"
            items = "".join(f"<item><instanceId>{i}</instanceId><instanceState><code>0</code><name>pending</name>"
                            f"</instanceState><instanceType>{f['InstanceType']}</instanceType></item>" for i in new)
            return f'<RunInstancesResponse xmlns="http://ec2.amazonaws.com/doc/2016-11-15/"><instancesSet>' \
                   f'{items}</instancesSet></RunInstancesResponse>'
        if act == "DescribeInstances":
            self.describe_count += 1
            if self.describe_count >= 2:                  # boxes come up on the second poll
                for i in self.instances:
                    if self.instances[i] == "pending":
                        self.instances[i] = "running"
            items = "".join(f"<item><instanceId>{i}</instanceId><instanceState><name>{s}</name></instanceState>"
                            f"<dnsName>{i}.compute.internal</dnsName></item>"
                            for i, s in self.instances.items() if i in ids)
            return f'<DescribeInstancesResponse xmlns="http://ec2.amazonaws.com/doc/2016-11-15/"><reservationSet>' \
                   f'<item><instancesSet>{items}</instancesSet></item></reservationSet></DescribeInstancesResponse>'
        if act == "TerminateInstances":
            items = ""
            for i in ids:
                items += (f"<item><instanceId>{i}</instanceId><currentState><name>shutting-down</name></currentState>"
                          f"<previousState><name>{self.instances[i]}</name></previousState></item>")
                self.instances[i] = "terminated"
            return f"<TerminateInstancesResponse><instancesSet>{items}</instancesSet></TerminateInstancesResponse>"
        if act == "RequestSpotInstances":
            assert f["LaunchSpecification.ImageId"] and f["SpotPrice"] == "0.05"
            return "<RequestSpotInstancesResponse><spotInstanceRequestSet><item><spotInstanceRequestId>sir-1" \
                   "</spotInstanceRequestId></item></spotInstanceRequestSet></RequestSpotInstancesResponse>"
        return "<Response><Errors><Error><Code>InvalidAction</Code><Message>nope</Message></Error></Errors></Response>"

    def emr(self, act, p):
        self.calls[-1] = act
        if act == "ListClusters":
            return 200, {"Clusters": [{"Id": k, "Name": v["Name"]} for k, v in self.clusters.items()
                                      if v["State"] in p["ClusterStates"]]}
        if act == "RunJobFlow":
            cid = f"j-{len(self.clusters)}"
            self.clusters[cid] = dict(p, State="STARTING")
            return 200, {"JobFlowId": cid}
        if act == "TerminateJobFlows":
            for c in p["JobFlowIds"]:
                self.clusters[c]["State"] = "TERMINATING"
            return 200, {}
        if act == "AddJobFlowSteps":
            sid = f"s-{len(self.steps)}"
            self.steps[sid] = {"step": p["Steps"][0], "polls": 0}
            return 200, {"StepIds": [sid]}
        if act == "DescribeStep":
            s = self.steps[p["StepId"]]
            s["polls"] += 1
            return 200, {"Step": {"Status": {"State": "RUNNING" if s["polls"] < 3 else "COMPLETED"}}}
        return 400, {"__type": "InvalidRequestException", "message": f"unknown {act}"}

    def close(self):
        self.srv.shutdown()


@pytest.fixture
def fake():
    f = FakeAws()
    yield f
    f.close()


def test_ec2_box_creator_life_cycle(fake):
    creds = C.Credentials(AK, SK)
    bc = aws.Ec2BoxCreator("ami-123", 3, "m5.large", "sg-1", "kp", endpoint=fake.url, credentials=creds, poll_s=0.01)
    ids = bc.create()
    assert ids == ["i-0000", "i-0001", "i-0002"] and bc.getBoxesCreated() == ids
    assert not bc.allRunning()
    bc.blockTillAllRunning(timeout_s=5)
    assert bc.getHosts() == [f"{i}.compute.internal" for i in ids]
    changes = bc.blowupBoxes()
    assert [c[0] for c in changes] == ids and all(c[1:] == ("running", "shutting-down") for c in changes)
    assert bc.createSpot("0.05") == ["sir-1"]
    with pytest.raises(C.AwsError, match="InvalidAction"):
        bc.getEc2().call("NoSuchAction")


def test_cluster_setup_provisions_every_host_and_starts_torchrun(fake):
    ran = []
    creds = C.Credentials(AK, SK)
    bc = aws.Ec2BoxCreator("ami-1", 2, "mi355x.48xlarge", endpoint=fake.url, credentials=creds, poll_s=0.01)
    cs = aws.ClusterSetup(bc, ["pip list"], keyFile="/k.pem", runner=lambda argv: (ran.append(argv), (0, ""))[1])
    hosts = cs.exec(script="train.py")
    assert len(hosts) == 2
    cmds = [a[-1] for a in ran]
    assert cmds[0] == "pip list" and cmds[1] == "pip list"
    assert "--node-rank 0" in cmds[2] and "--node-rank 1" in cmds[3]
    assert all(f"--master-addr {hosts[0]}" in c for c in cmds[2:])
    assert ran[0][:1] == ["ssh"] and "-i" in ran[0] and "/k.pem" in ran[0]


def test_host_provisioner_upload_and_run(tmp_path):
    ran = []
    script = tmp_path / "setup.sh"
    script.write_text("echo hi")
    hp = aws.HostProvisioner("h1", "me", runner=lambda argv: (ran.append(argv), (0, "ok"))[1])
    hp.uploadAndRun(str(script), "/opt/job")
    assert ran[0][0] == "ssh" and ran[0][-1] == "mkdir -p /opt/job"
    assert ran[1][0] == "scp" and ran[1][-1] == "me@h1:/opt/job/setup.sh"
    assert ran[2][-1].startswith("cd /opt/job && chmod +x /opt/job/setup.sh")
    bad = aws.HostProvisioner("h1", runner=lambda argv: (1, "denied"))
    with pytest.raises(RuntimeError, match="denied"):
        bad.runRemoteCommand("true")


def test_emr_client_cluster_and_step(fake, tmp_path, monkeypatch):
    monkeypatch.setenv("DL4J_AMD_S3_ROOT", str(tmp_path / "s3"))
    (tmp_path / "s3" / "jobs").mkdir(parents=True)
    creds = C.Credentials(AK, SK)
    cli = (aws.SparkEMRClient.Builder().clusterName("train").instanceCount(3).instanceType("g")
           .instanceBidPrice(1.5).emrConfigs([aws.EmrConfig("spark", {"a": "b"})]).s3JarFolder("s3://jobs/bin")
           .endpointUrl(fake.url).awsCredentials(creds).pollSeconds(0.01).build())
    cid = cli.createCluster()
    req = fake.clusters[cid]
    assert req["Instances"]["InstanceGroups"][1] == {"Name": "core", "InstanceRole": "CORE", "InstanceType": "g",
                                                     "InstanceCount": 2, "Market": "SPOT", "BidPrice": "1.5"}
    assert req["Configurations"] == [{"Classification": "spark", "Properties": {"a": "b"}}]
    assert cli.listActiveClusterNames() == ["train"] and cli.listActiveClusterIds() == [cid]
    with pytest.raises(RuntimeError, match="already deployed"):
        cli.createCluster()
    script = tmp_path / "train.py"
    script.write_text("print(1)")
    sid = cli.submitJob(str(script), ["--epochs", 2])
    args = fake.steps[sid]["step"]["HadoopJarStep"]["Args"]
    assert args[:3] == ["python3", "-m", "torch.distributed.run"] and "--nnodes=3" in args
    assert args[-3:] == ["s3://jobs/bin/train.py", "--epochs", "2"]
    assert (tmp_path / "s3" / "jobs" / "bin" / "train.py").read_text() == "print(1)"
    assert cli.checkStatus() == "COMPLETED"
    assert cli.terminateCluster() == cid and cli.listActiveClusterIds() == []
