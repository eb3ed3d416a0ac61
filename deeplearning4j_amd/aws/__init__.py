"""Cloud storage / provisioning helpers (replacement for deeplearning4j-aws, SURVEY §2.9:
``BaseS3`` credentials (s3/BaseS3.java:64-71), ``S3Uploader`` / ``S3Downloader`` / ``BucketIterator`` /
``BaseS3DataSetIterator`` (s3/reader/*), ``DataSetLoader``, EC2 ``Ec2BoxCreator`` / ``ClusterSetup`` /
``HostProvisioner`` and the EMR Spark client).

Object storage goes through ``boto3`` when it is importable. This image has no boto3 and no network, so an
S3-compatible local object store is built in: set ``DL4J_AMD_S3_ROOT`` (or pass ``root=``) and ``s3://bucket/key``
maps to ``<root>/bucket/key`` with the same API — the path used by the tests and by air-gapped clusters that mount
a shared filesystem. Provisioning (EC2 box creation, SSH host provisioning, the EMR cluster client) talks to
the AWS APIs directly through the SigV4 client in :mod:`.client` (no SDK needed; endpoints are configurable so
the tests run against a local fake service).
"""
import io
import os
import shutil


class AwsUnavailable(RuntimeError):
    pass


def _boto3():
    try:
        import boto3  # noqa: F401
        return boto3
    except ImportError:
        return None


class BaseS3:
    """Credentials from AWS_ACCESS_KEY_ID / AWS_SECRET_ACCESS_KEY (or the constructor); backend = boto3 client or the
    local object store rooted at ``root`` / $DL4J_AMD_S3_ROOT."""

    def __init__(self, accessKey=None, secretKey=None, root=None, endpoint=None):
        self.accessKey = accessKey or os.environ.get("AWS_ACCESS_KEY_ID") or os.environ.get("AWS_ACCESS_KEY")
        self.secretKey = secretKey or os.environ.get("AWS_SECRET_ACCESS_KEY") or os.environ.get("AWS_SECRET_KEY")
        self.root = root or os.environ.get("DL4J_AMD_S3_ROOT")
        self.client = None
        if self.root is None:
            b3 = _boto3()
            if b3 is None:
                raise AwsUnavailable("boto3 is not installed and no local object store root is configured "
                                     "(set DL4J_AMD_S3_ROOT)")
            self.client = b3.client("s3", aws_access_key_id=self.accessKey, aws_secret_access_key=self.secretKey,
                                    endpoint_url=endpoint)

    # ---------------------------------------------------------------- local object store
    def _path(self, bucket, key=""):
        p = os.path.realpath(os.path.join(self.root, bucket, key))
        if not p.startswith(os.path.realpath(self.root)):
            raise ValueError(f"key escapes the object store: {bucket}/{key}")
        return p

    def buckets(self):
        if self.client is not None:
            return [b["Name"] for b in self.client.list_buckets()["Buckets"]]
        return sorted(d for d in os.listdir(self.root) if os.path.isdir(os.path.join(self.root, d)))

    def createBucket(self, bucket):
        if self.client is not None:
            self.client.create_bucket(Bucket=bucket)
        else:
            os.makedirs(self._path(bucket), exist_ok=True)

    def keysForBucket(self, bucket):
        if self.client is not None:
            keys, token = [], None
            while True:
                kw = dict({"Bucket": bucket}, **({"ContinuationToken": token} if token else {}))
                r = self.client.list_objects_v2(**kw)
                keys += [o["Key"] for o in r.get("Contents", [])]
                if not r.get("IsTruncated"):
                    return keys
                token = r["NextContinuationToken"]
        base = self._path(bucket)
        out = []
        for d, _, files in os.walk(base):
            for f in files:
                out.append(os.path.relpath(os.path.join(d, f), base).replace(os.sep, "/"))
        return sorted(out)


class S3Uploader(BaseS3):
    def upload(self, file, bucket, key=None):
        key = key or os.path.basename(file)
        if self.client is not None:
            self.client.upload_file(file, bucket, key)
        else:
            dst = self._path(bucket, key)
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            shutil.copyfile(file, dst)
        return f"s3://{bucket}/{key}"

    multiPartUpload = upload

    def uploadBytes(self, data, bucket, key):
        if self.client is not None:
            self.client.put_object(Bucket=bucket, Key=key, Body=data)
        else:
            dst = self._path(bucket, key)
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            with open(dst, "wb") as fh:
                fh.write(data)


class S3Downloader(BaseS3):
    def download(self, bucket, key, dest):
        if self.client is not None:
            self.client.download_file(bucket, key, dest)
        else:
            shutil.copyfile(self._path(bucket, key), dest)
        return dest

    def objectForKey(self, bucket, key):
        """Stream (file-like) of an object."""
        if self.client is not None:
            return io.BytesIO(self.client.get_object(Bucket=bucket, Key=key)["Body"].read())
        return open(self._path(bucket, key), "rb")

    def iterateBucket(self, bucket):
        return BucketIterator(bucket, self)

    def paginate(self, bucket, keys_per_page=1000):
        keys = self.keysForBucket(bucket)
        for i in range(0, len(keys), keys_per_page):
            yield keys[i:i + keys_per_page]


class BucketIterator:
    """Iterates the objects of a bucket as file-like streams (s3/reader/BucketIterator.java)."""

    def __init__(self, bucket, downloader=None):
        self.bucket = bucket
        self.s3 = downloader or S3Downloader()
        self.keys = self.s3.keysForBucket(bucket)
        self._i = 0

    def hasNext(self):
        return self._i < len(self.keys)

    def next(self):
        k = self.keys[self._i]
        self._i += 1
        return self.s3.objectForKey(self.bucket, k)

    def reset(self):
        self._i = 0

    def __iter__(self):
        self.reset()
        while self.hasNext():
            yield self.next()


class DataSetLoader:
    """Loads a DataSet saved with ``DataSet.save`` from a stream (aws/dataset/DataSetLoader.java)."""

    @staticmethod
    def load(stream):
        from ..datasets import DataSet
        return DataSet.load(stream)


class BaseS3DataSetIterator:
    """DataSetIterator over a bucket of serialized DataSets (one object per minibatch)."""

    def __init__(self, bucket, downloader=None):
        self.it = BucketIterator(bucket, downloader)

    def hasNext(self):
        return self.it.hasNext()

    def next(self):
        with self.it.next() as fh:
            return DataSetLoader.load(io.BytesIO(fh.read()))

    def reset(self):
        self.it.reset()

    def __iter__(self):
        self.reset()
        while self.hasNext():
            yield self.next()


def save_dataset_to_bucket(ds, bucket, key, uploader=None):
    """Serialize a DataSet into the object store (the producer side of BaseS3DataSetIterator)."""
    buf = io.BytesIO()
    ds.save(buf)
    (uploader or S3Uploader()).uploadBytes(buf.getvalue(), bucket, key)


# ------------------------------------------------------------------------------------------------ provisioning
def _ec2(region, endpoint, credentials):
    from .client import Ec2Client
    return Ec2Client(region=region, endpoint=endpoint, credentials=credentials)


class Ec2BoxCreator:
    """Launch, watch and terminate EC2 training hosts (ec2/Ec2BoxCreator.java:58-215) over the SigV4 Query client
    in :mod:`.client` (boto3 is not needed). ``endpoint`` / ``credentials`` default to the AWS environment."""
    DEFAULT_AMI = "ami-8997afe0"

    def __init__(self, amiId=None, numBoxes=1, size="m5.large", securityGroupId=None, keyPair=None,
                 region="us-east-1", endpoint=None, credentials=None, poll_s=1.0):
        self.amiId = amiId or self.DEFAULT_AMI
        self.numBoxes, self.size = int(numBoxes), size
        self.securityGroupId, self.keyPair, self.region = securityGroupId, keyPair, region
        self.endpoint, self.credentials, self.poll_s = endpoint, credentials, poll_s
        self.instanceIds = []
        self.spotRequestIds = []
        self._client = None

    def getEc2(self):
        if self._client is None:
            self._client = _ec2(self.region, self.endpoint, self.credentials)
        return self._client

    def setRegion(self, region):
        self.region, self._client = region, None

    def _spec(self):
        kw = {"ImageId": self.amiId, "InstanceType": self.size}
        if self.keyPair:
            kw["KeyName"] = self.keyPair
        if self.securityGroupId:
            kw["SecurityGroupId"] = [self.securityGroupId]
        return kw

    def create(self):
        """RunInstances(MinCount=1, MaxCount=numBoxes); a second call first terminates the previous boxes, as the
        reference does (Ec2BoxCreator.java:130-154)."""
        if self.instanceIds:
            self.blowupBoxes()
        ec2 = self.getEc2()
        root = ec2.call("RunInstances", MinCount=1, MaxCount=self.numBoxes, **self._spec())
        self.instanceIds = [i["id"] for i in ec2.instances(root)]
        return list(self.instanceIds)

    def createSpot(self, spotPrice="0.03", count=None):
        """RequestSpotInstances with this creator's launch specification (Ec2BoxCreator.java:79-120)."""
        root = self.getEc2().call("RequestSpotInstances", SpotPrice=str(spotPrice),
                                  InstanceCount=int(count or self.numBoxes), LaunchSpecification=self._spec())
        self.spotRequestIds = [e.text for e in root.iter("spotInstanceRequestId")]
        return list(self.spotRequestIds)

    def blowupBoxes(self):
        """TerminateInstances on every box this creator launched; returns [(id, previous, current)] state changes."""
        if not self.instanceIds:
            return []
        root = self.getEc2().call("TerminateInstances", InstanceId=list(self.instanceIds))
        out = []
        for it in root.iter("item"):
            if it.findtext("instanceId") and it.find("currentState") is not None:
                out.append((it.findtext("instanceId"), it.find("previousState").findtext("name"),
                            it.find("currentState").findtext("name")))
        return out

    def _describe(self):
        ec2 = self.getEc2()
        return [i for i in ec2.instances(ec2.call("DescribeInstances", InstanceId=list(self.instanceIds)))
                if i["id"] in self.instanceIds]

    def allRunning(self):
        """True when every launched box is ``running`` (terminated boxes, state code 48, are ignored as in
        Ec2BoxCreator.java:177-198)."""
        if not self.instanceIds:
            return False
        return all(i["state"] in ("running", "terminated") for i in self._describe())

    def blockTillAllRunning(self, timeout_s=900.0):
        import time
        t0 = time.monotonic()
        while not self.allRunning():
            if time.monotonic() - t0 > timeout_s:
                raise TimeoutError(f"EC2 boxes not running after {timeout_s:.0f} s: {self.instanceIds}")
            time.sleep(self.poll_s)

    def getHosts(self):
        """Public DNS names (private IP when there is none) of the launched boxes."""
        return [i["publicDns"] or i["privateIp"] for i in self._describe()]

    def getBoxesCreated(self):
        return list(self.instanceIds)


class HostProvisioner:
    """Upload files to a host and run commands on it (ec2/provision/HostProvisioner.java:53-270) through the
    system ``ssh`` / ``scp`` clients. ``runner`` (argv list -> (returncode, output)) replaces the subprocess call,
    e.g. for dry runs or tests."""

    def __init__(self, host, user="ubuntu", password=None, port=22, keyFile=None, runner=None):
        if password:
            raise ValueError("password authentication is not supported; use a key file (addKeyFile)")
        self.host, self.user, self.port, self.keyFile = host, user, int(port), keyFile
        self.runner = runner or self._subprocess

    @staticmethod
    def _subprocess(argv):
        import subprocess
        r = subprocess.run(argv, capture_output=True, text=True)
        return r.returncode, r.stdout + r.stderr

    def addKeyFile(self, keyFile):
        self.keyFile = keyFile

    def _opts(self, port_flag):
        o = ["-o", "StrictHostKeyChecking=accept-new", "-o", "BatchMode=yes", port_flag, str(self.port)]
        if self.keyFile:
            o += ["-i", self.keyFile]
        return o

    def _run(self, argv):
        rc, out = self.runner(argv)
        if rc != 0:
            raise RuntimeError(f"{argv[0]} on {self.host} failed ({rc}): {out.strip()[-500:]}")
        return out

    def runRemoteCommand(self, remoteCommand):
        import shlex
        return self._run(["ssh"] + self._opts("-p") + [f"{self.user}@{self.host}", remoteCommand]
                         if isinstance(remoteCommand, str) else
                         ["ssh"] + self._opts("-p") + [f"{self.user}@{self.host}", shlex.join(remoteCommand)])

    def uploadForDeployment(self, src, dest):
        """Copy a file or directory (recursively) to ``dest`` on the host, creating the parent directory."""
        import shlex
        self.runRemoteCommand(f"mkdir -p {shlex.quote(os.path.dirname(dest.rstrip('/')) or '.')}")
        flags = ["-r"] if os.path.isdir(src) else []
        return self._run(["scp"] + flags + self._opts("-P") + [src, f"{self.user}@{self.host}:{dest}"])

    def uploadAndRun(self, script, rootDir):
        """Upload ``script`` into ``rootDir`` and execute it there (HostProvisioner.java:92-99)."""
        import shlex
        dest = os.path.join(rootDir, os.path.basename(script))
        self.uploadForDeployment(script, dest)
        return self.runRemoteCommand(f"cd {shlex.quote(rootDir)} && chmod +x {shlex.quote(dest)} && "
                                     f"./{shlex.quote(os.path.basename(script))}")


class ClusterSetup:
    """Provision a training cluster (ec2/provision/ClusterSetup.java): launch the boxes, wait until they run, run
    the per-host setup commands, then start one ``torch.distributed.run`` per host (one rank per MI355X; node 0
    is the rendezvous master) — the replacement for the reference's Spark/Aeron worker bootstrap."""

    def __init__(self, creator, setupCommands=(), user="ubuntu", keyFile=None, runner=None, gpusPerHost=8):
        self.creator = creator
        self.setupCommands = list(setupCommands)
        self.user, self.keyFile, self.runner, self.gpusPerHost = user, keyFile, runner, int(gpusPerHost)

    def launch_command(self, nnodes, master_addr, port=29500, script="train.py", node_rank=None):
        rank = "" if node_rank is None else f"--node-rank {node_rank} "
        return (f"python -m torch.distributed.run --nnodes {nnodes} {rank}--nproc-per-node {self.gpusPerHost} "
                f"--master-addr {master_addr} --master-port {port} {script}")

    def provisioners(self, hosts):
        return [HostProvisioner(h, self.user, keyFile=self.keyFile, runner=self.runner) for h in hosts]

    def exec(self, script=None, port=29500):
        """Launch + wait + set up every host; with ``script`` also start training. Returns the host list."""
        self.creator.create()
        self.creator.blockTillAllRunning()
        hosts = self.creator.getHosts()
        provs = self.provisioners(hosts)
        for p in provs:
            for c in self.setupCommands:
                p.runRemoteCommand(c)
        if script is not None:
            for r, p in enumerate(provs):
                p.runRemoteCommand("nohup " + self.launch_command(len(hosts), hosts[0], port, script, r)
                                   + " > train.log 2>&1 &")
        return hosts


class EmrConfig:
    """One EMR configuration classification (emr/EmrConfig.java): ``classification`` + ``properties``."""

    def __init__(self, classification, properties=None, configs=None):
        self.classification, self.properties, self.configs = classification, dict(properties or {}), configs or []

    def toAws(self):
        d = {"Classification": self.classification, "Properties": self.properties}
        if self.configs:
            d["Configurations"] = [c.toAws() for c in self.configs]
        return d


class SparkEMRClient:
    """EMR cluster life cycle + job submission (emr/SparkEMRClient.java:58-250) over the SigV4 JSON client.
    Differences by design: the submitted step runs ``torch.distributed.run`` on the cluster's GPU nodes through
    EMR's ``command-runner.jar`` instead of ``spark-submit`` of an uber jar, and the training script is uploaded
    through this package's object store (``S3Uploader``) when ``s3JarFolder`` is set."""
    ACTIVE_STATES = ["RUNNING", "STARTING", "WAITING", "BOOTSTRAPPING"]

    def __init__(self, b):
        self.__dict__.update(b.v)
        self.clusterId = self.lastStepId = None
        from .client import EmrClient
        self._emr = EmrClient(region=self.region, endpoint=self.endpoint, credentials=self.credentials)

    class Builder:
        """Fluent builder; the values live in ``self.v`` so the setter names can match the reference's."""
        _FIELDS = {"clusterName": "clusterName", "awsRegion": "region", "emrRelease": "releaseLabel",
                   "emrServiceRole": "serviceRole", "emrConfigs": "configs", "subnetId": "subnetId",
                   "securityGroupIDs": "securityGroupIds", "instanceCount": "instanceCount",
                   "instanceType": "instanceType", "instanceBidPrice": "bidPrice", "instanceRole": "instanceRole",
                   "s3JarFolder": "s3JarFolder", "sparkTimeOutDurationMinutes": "timeoutMinutes",
                   "endpointUrl": "endpoint", "awsCredentials": "credentials", "pollSeconds": "poll_s"}

        def __init__(self):
            self.v = {"clusterName": "dl4j-amd-cluster", "region": "us-east-1", "releaseLabel": "emr-7.2.0",
                      "serviceRole": "EMR_DefaultRole", "instanceRole": "EMR_EC2_DefaultRole", "configs": [],
                      "subnetId": None, "securityGroupIds": [], "instanceCount": 1, "instanceType": "m5.xlarge",
                      "bidPrice": None, "s3JarFolder": None, "timeoutMinutes": 90, "endpoint": None,
                      "credentials": None, "poll_s": 10.0}

        def __getattr__(self, name):
            field = SparkEMRClient.Builder._FIELDS.get(name)
            if field is None:
                raise AttributeError(name)

            def setter(value):
                if field in ("configs", "securityGroupIds"):
                    value = list(value)
                elif field in ("instanceCount", "timeoutMinutes"):
                    value = int(value)
                self.v[field] = value
                return self
            return setter

        def build(self):
            return SparkEMRClient(self)

    def _run_job_flow_request(self):
        groups = [{"Name": "master", "InstanceRole": "MASTER", "InstanceType": self.instanceType,
                   "InstanceCount": 1}]
        if self.instanceCount > 1:
            core = {"Name": "core", "InstanceRole": "CORE", "InstanceType": self.instanceType,
                    "InstanceCount": self.instanceCount - 1}
            if self.bidPrice is not None:
                core["Market"], core["BidPrice"] = "SPOT", str(self.bidPrice)
            groups.append(core)
        inst = {"InstanceGroups": groups, "KeepJobFlowAliveWhenNoSteps": True}
        if self.subnetId:
            inst["Ec2SubnetId"] = self.subnetId
        if self.securityGroupIds:
            inst["AdditionalMasterSecurityGroups"] = list(self.securityGroupIds)
            inst["AdditionalSlaveSecurityGroups"] = list(self.securityGroupIds)
        return {"Name": self.clusterName, "ReleaseLabel": self.releaseLabel, "ServiceRole": self.serviceRole,
                "JobFlowRole": self.instanceRole, "Instances": inst, "VisibleToAllUsers": True,
                "Configurations": [c.toAws() for c in self.configs]}

    def _clusters(self):
        return self._emr.call("ListClusters", ClusterStates=list(self.ACTIVE_STATES)).get("Clusters", [])

    def _find(self):
        for c in self._clusters():
            if c.get("Name") == self.clusterName:
                return c
        return None

    def createCluster(self):
        c = self._find()
        if c is not None:
            raise RuntimeError(f"A cluster with name {self.clusterName} and id {c['Id']} is already deployed")
        self.clusterId = self._emr.call("RunJobFlow", **self._run_job_flow_request())["JobFlowId"]
        return self.clusterId

    def listActiveClusterNames(self):
        return [c["Name"] for c in self._clusters()]

    def listActiveClusterIds(self):
        return [c["Id"] for c in self._clusters()]

    def terminateCluster(self):
        c = self._find()
        if c is None:
            return None
        self._emr.call("TerminateJobFlows", JobFlowIds=[c["Id"]])
        return c["Id"]

    def submitJob(self, script, args=(), nprocPerNode=8, uploader=None):
        """Upload the training script (when ``s3JarFolder`` is set) and add one EMR step that runs it under
        ``torch.distributed.run`` on the cluster; returns the step id."""
        c = self._find()
        if c is None:
            raise RuntimeError(f"no active cluster named {self.clusterName}")
        target = script
        if self.s3JarFolder:
            bucket, _, prefix = self.s3JarFolder.replace("s3://", "").partition("/")
            key = (prefix.rstrip("/") + "/" if prefix else "") + os.path.basename(script)
            with open(script, "rb") as f:
                (uploader or S3Uploader()).uploadBytes(f.read(), bucket, key)
            target = f"s3://{bucket}/{key}"
        argv = ["python3", "-m", "torch.distributed.run", f"--nnodes={self.instanceCount}",
                f"--nproc-per-node={int(nprocPerNode)}", target] + [str(a) for a in args]
        step = {"Name": f"dl4j-amd {os.path.basename(script)}", "ActionOnFailure": "CONTINUE",
                "HadoopJarStep": {"Jar": "command-runner.jar", "Args": argv}}
        r = self._emr.call("AddJobFlowSteps", JobFlowId=c["Id"], Steps=[step])
        self.lastStepId = r["StepIds"][0]
        return self.lastStepId

    def checkStatus(self, stepId=None):
        """Poll the step until it leaves PENDING/RUNNING or the timeout passes; returns the final state
        (SparkEMRClient.java:202-237)."""
        import time
        c = self._find()
        sid = stepId or self.lastStepId
        t0 = time.monotonic()
        while True:
            st = self._emr.call("DescribeStep", ClusterId=c["Id"], StepId=sid)["Step"]["Status"]["State"]
            if st not in ("PENDING", "RUNNING"):
                return st
            if time.monotonic() - t0 > 60.0 * self.timeoutMinutes:
                raise TimeoutError(f"step {sid} still {st} after {self.timeoutMinutes} min")
            time.sleep(self.poll_s)
