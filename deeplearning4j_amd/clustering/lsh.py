"""Random-projection LSH for cosine distance (RandomProjectionLSH.java).

Hash = sign(x @ R) with R ~ N(0, 1/sqrt(inDimension)) of shape [inDimension, hashLength]; a data point is in the
query's bucket when all hash bits match. With numTables > 1 the query is additionally perturbed numTables times by
unit noise scaled by ``radius`` ("entropy" probes) and the buckets are OR-ed. All of it is batched GEMM/compare on
the device the index lives on.
"""
import torch


class RandomProjectionLSH:
    def __init__(self, hashLength, numTables, inDimension, radius, rng=None, device=None):
        self.hashLength, self.numTables, self.inDimension, self.radius = hashLength, numTables, inDimension, radius
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.gen = rng if isinstance(rng, torch.Generator) else torch.Generator().manual_seed(
            12345 if rng is None else int(rng))
        self.randomProjection = (torch.randn(inDimension, hashLength, generator=self.gen) /
                                 inDimension ** 0.5).to(self.device)
        self.index = self.indexData = None

    def getDistanceMeasure(self):
        return "cosinedistance"

    def hash(self, data):
        data = torch.as_tensor(data, dtype=torch.float32, device=self.device)
        if data.dim() == 1:
            data = data.reshape(1, -1)
        if data.shape[1] != self.inDimension:
            raise ValueError(f"Invalid shape {tuple(data.shape)}: this table expects dimension {self.inDimension}")
        return torch.sign(data @ self.randomProjection)

    def makeIndex(self, data):
        self.indexData = torch.as_tensor(data, dtype=torch.float32, device=self.device)
        self.index = self.hash(self.indexData)

    def entropy(self, query):
        q = torch.as_tensor(query, dtype=torch.float32, device=self.device).reshape(1, -1)
        noise = (torch.randn(self.numTables, self.inDimension, generator=self.gen) * self.radius).to(self.device)
        noise = noise / noise.norm(dim=1, keepdim=True).clamp_min(1e-30)
        return noise + q

    def bucket(self, query):
        """0/1 mask [N] of indexed points sharing a bucket with the query (or any entropy probe)."""
        probes = self.hash(query)
        if self.numTables > 1:
            probes = torch.cat([probes, self.hash(self.entropy(query))])
        match = (self.index.unsqueeze(0) == probes.unsqueeze(1)).all(-1)      # [probes, N]
        return match.any(0).float()

    def _bucket_data(self, query):
        m = self.bucket(query).bool()
        return self.indexData[m]

    def _sorted(self, query):
        data = self._bucket_data(query)
        if data.shape[0] == 0:
            return data, data.new_zeros(0)
        q = torch.as_tensor(query, dtype=torch.float32, device=self.device).reshape(1, -1)
        d = 1.0 - torch.nn.functional.cosine_similarity(data, q, dim=1)
        order = torch.argsort(d)
        return data[order], d[order]

    def search(self, query, k_or_range):
        if isinstance(k_or_range, int):
            if k_or_range < 1:
                raise ValueError("An ANN search for k neighbors should at least seek one neighbor")
            data, _ = self._sorted(query)
            return data[:k_or_range]
        if k_or_range < 0:
            raise ValueError("ANN search should have a positive maximum search radius")
        data, d = self._sorted(query)
        return data[d <= k_or_range]
