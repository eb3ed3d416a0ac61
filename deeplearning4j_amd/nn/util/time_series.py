"""Time-series helpers (reference nn/util/TimeSeriesUtils.java:149,188 — reverse with/without mask)."""
import torch


def reverse_time_series(x, mask=None):
    """Reverse along the time axis (dim 2 for [mb, size, T]; dim 1 for [mb, T] masks). With a mask,
    each example's valid (mask==1, left-aligned) prefix is reversed in place and padding stays put."""
    tdim = x.dim() - 1
    if mask is None:
        if x.is_cuda:
            from deeplearning4j_amd.ops import nd4j_kernels
            r = nd4j_kernels.reverse(x, [tdim])                    # negative-stride copy kernel (nd4j_ops.hip)
            if r is not None:
                return r
        return torch.flip(x, [tdim])
    T = x.shape[tdim]
    lengths = mask.reshape(mask.shape[0], -1).sum(dim=1).long()            # [mb]
    t = torch.arange(T, device=x.device).unsqueeze(0)                       # [1, T]
    src = torch.where(t < lengths.unsqueeze(1), lengths.unsqueeze(1) - 1 - t, t)  # [mb, T]
    if x.dim() == 3:
        idx = src.unsqueeze(1).expand(x.shape[0], x.shape[1], T)
    else:
        idx = src
    return torch.gather(x, tdim, idx)


def last_time_step(x, mask=None):
    if mask is None:
        return x[:, :, -1]
    lengths = mask.reshape(mask.shape[0], -1).sum(dim=1).long().clamp(min=1)
    return x[torch.arange(x.shape[0], device=x.device), :, lengths - 1]


class TimeSeriesUtils:
    """Static helpers with the reference's names (nn/util/TimeSeriesUtils.java). 2-D forms of [mb, n, T] series are
    time-major (row t*mb + i is example i at step t), the layout RnnToFeedForwardPreProcessor produces."""

    @staticmethod
    def movingAverage(x, n):
        """Mean of every window of n consecutive values of a vector (len(x) - n + 1 values)."""
        x = torch.as_tensor(x).reshape(-1).double()
        c = torch.cumsum(x, 0)
        c[n:] = c[n:] - c[:-n].clone()
        return c[n - 1:] / n

    @staticmethod
    def reverseTimeSeries(x, mask=None):
        return reverse_time_series(x, mask)

    @staticmethod
    def reshape3dTo2d(x):
        mb, n, T = x.shape
        return x.permute(2, 0, 1).reshape(T * mb, n)

    @staticmethod
    def reshape2dTo3d(x, miniBatchSize):
        rows, n = x.shape
        return x.reshape(rows // miniBatchSize, miniBatchSize, n).permute(1, 2, 0)

    @staticmethod
    def reshapeTimeSeriesMaskToVector(mask):
        return mask.t().reshape(-1, 1)

    @staticmethod
    def reshapeVectorToTimeSeriesMask(v, miniBatchSize):
        return v.reshape(-1, miniBatchSize).t()

    @staticmethod
    def pullLastTimeSteps(x, mask=None):
        return last_time_step(x, mask)
