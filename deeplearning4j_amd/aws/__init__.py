"""Cloud storage / provisioning helpers (replacement for deeplearning4j-aws, SURVEY §2.9:
``BaseS3`` credentials (s3/BaseS3.java:64-71), ``S3Uploader`` / ``S3Downloader`` / ``BucketIterator`` /
``BaseS3DataSetIterator`` (s3/reader/*), ``DataSetLoader``, EC2 ``Ec2BoxCreator`` / ``ClusterSetup`` /
``HostProvisioner`` and the EMR Spark client).

Object storage goes through ``boto3`` when it is importable. This image has no boto3 and no network, so an
S3-compatible local object store is built in: set ``DL4J_AMD_S3_ROOT`` (or pass ``root=``) and ``s3://bucket/key``
maps to ``<root>/bucket/key`` with the same API — the path used by the tests and by air-gapped clusters that mount
a shared filesystem. Provisioning (EC2 / EMR) needs the AWS SDK and network; without them those classes raise
:class:`AwsUnavailable` with the reason, instead of failing later.
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
class Ec2BoxCreator:
    """Launch EC2 instances (ec2/Ec2BoxCreator.java). Needs boto3 + network."""

    def __init__(self, amiId, numBoxes, size, securityGroupId=None, keyPair=None, region="us-east-1"):
        self.amiId, self.numBoxes, self.size = amiId, int(numBoxes), size
        self.securityGroupId, self.keyPair, self.region = securityGroupId, keyPair, region
        self.instanceIds = []

    def create(self):
        b3 = _boto3()
        if b3 is None:
            raise AwsUnavailable("Ec2BoxCreator needs boto3 and network access (not available in this image)")
        ec2 = b3.client("ec2", region_name=self.region)
        kw = {"ImageId": self.amiId, "MinCount": self.numBoxes, "MaxCount": self.numBoxes, "InstanceType": self.size}
        if self.keyPair:
            kw["KeyName"] = self.keyPair
        if self.securityGroupId:
            kw["SecurityGroupIds"] = [self.securityGroupId]
        r = ec2.run_instances(**kw)
        self.instanceIds = [i["InstanceId"] for i in r["Instances"]]
        return self.instanceIds

    def blockTillAllRunning(self):
        b3 = _boto3()
        if b3 is None:
            raise AwsUnavailable("boto3 unavailable")
        b3.client("ec2", region_name=self.region).get_waiter("instance_running").wait(InstanceIds=self.instanceIds)


class ClusterSetup:
    """Provision a training cluster: boxes + per-host setup; each host then runs
    ``torchrun --nnodes N --nproc-per-node 8`` (one rank per MI355X) — the replacement for the reference's
    Spark/Aeron worker bootstrap (ec2/provision/ClusterSetup.java)."""

    def __init__(self, creator, setupCommands=()):
        self.creator = creator
        self.setupCommands = list(setupCommands)

    def launch_command(self, nnodes, master_addr, port=29500, script="train.py"):
        return (f"python -m torch.distributed.run --nnodes {nnodes} --nproc-per-node 8 --master-addr {master_addr} "
                f"--master-port {port} {script}")

    def exec(self):
        ids = self.creator.create()
        self.creator.blockTillAllRunning()
        return ids


class SparkEMRClient:
    """EMR cluster client of the reference (emr/SparkEMRClient.java): not applicable without Spark/EMR; the
    distributed front end here is :mod:`deeplearning4j_amd.parallel.cluster` over torch.distributed."""

    def __init__(self, *a, **kw):
        raise AwsUnavailable("EMR/Spark is replaced by torch.distributed training masters "
                             "(deeplearning4j_amd.parallel.cluster); no EMR client in this build")

