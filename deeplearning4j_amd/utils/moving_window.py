"""MovingWindowMatrix: split a matrix into consecutive windowRows x windowCols windows, optionally with their three
rotations (reference deeplearning4j-nn/src/main/java/org/deeplearning4j/util/MovingWindowMatrix.java). Windows are
successive runs of windowRows*windowCols elements of the row-major flattening; an incomplete tail is dropped."""
import torch


class MovingWindowMatrix:
    def __init__(self, toSlice, windowRowSize, windowColumnSize, addRotate=False):
        self.toSlice = torch.as_tensor(toSlice)
        self.windowRowSize, self.windowColumnSize = int(windowRowSize), int(windowColumnSize)
        self.addRotate = bool(addRotate)

    def windows(self, flattened=False):
        flat = self.toSlice.reshape(-1)
        k = self.windowRowSize * self.windowColumnSize
        out = []
        for start in range(0, flat.numel() - k + 1, k):
            w = flat[start:start + k].clone()
            w = w if flattened else w.reshape(self.windowRowSize, self.windowColumnSize)
            if self.addRotate:
                sq = w.reshape(self.windowRowSize, self.windowColumnSize)
                for r in (1, 2, 3):                    # 90, 180, 270 degrees, then the window itself
                    rot = torch.rot90(sq, r, dims=(0, 1))
                    out.append(rot.reshape(-1) if flattened else rot)
            out.append(w)
        return out
