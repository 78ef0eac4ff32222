"""Block grid with halos: the nifty.tools.blocking semantics the watershed path uses
(watershed.py:252-264, :365; utils/volume_utils.py:52-88, :142-205).

Block ids are C-order over the block grid; blocks at the upper volume edge are clipped;
outer blocks (block + halo) are clipped to the volume.
"""
import numpy as np


class Block:
    def __init__(self, begin, end):
        self.begin = list(begin)
        self.end = list(end)
        self.shape = [e - b for b, e in zip(self.begin, self.end)]

    def __repr__(self):
        return 'Block(%r, %r)' % (self.begin, self.end)


class BlockWithHalo:
    def __init__(self, outer, inner, inner_local):
        self.outerBlock = outer
        self.innerBlock = inner
        self.innerBlockLocal = inner_local


class Blocking:
    def __init__(self, roiBegin, roiEnd, blockShape):
        self.roiBegin = [int(r) for r in roiBegin]
        self.roiEnd = [int(r) for r in roiEnd]
        self.blockShape = [int(b) for b in blockShape]
        self.ndim = len(self.blockShape)
        self.blocksPerAxis = [int(np.ceil((e - b) / float(s)))
                              for b, e, s in zip(self.roiBegin, self.roiEnd, self.blockShape)]
        self.numberOfBlocks = int(np.prod(self.blocksPerAxis))
        strides = [1] * self.ndim
        for d in range(self.ndim - 2, -1, -1):
            strides[d] = strides[d + 1] * self.blocksPerAxis[d + 1]
        self._strides = strides

    def blockCoordinates(self, block_id):
        return [(block_id // s) % n for s, n in zip(self._strides, self.blocksPerAxis)]

    def coordinatesToBlockId(self, coords):
        bc = [(int(c) - b) // s for c, b, s in zip(coords, self.roiBegin, self.blockShape)]
        return int(sum(c * s for c, s in zip(bc, self._strides)))

    def getBlock(self, block_id):
        c = self.blockCoordinates(block_id)
        begin = [b + ci * s for b, ci, s in zip(self.roiBegin, c, self.blockShape)]
        end = [min(bb + s, e) for bb, s, e in zip(begin, self.blockShape, self.roiEnd)]
        return Block(begin, end)

    def getBlockWithHalo(self, block_id, halo):
        inner = self.getBlock(block_id)
        ob = [max(b - h, r) for b, h, r in zip(inner.begin, halo, self.roiBegin)]
        oe = [min(e + h, r) for e, h, r in zip(inner.end, halo, self.roiEnd)]
        outer = Block(ob, oe)
        local = Block([b - o for b, o in zip(inner.begin, ob)], [e - o for e, o in zip(inner.end, ob)])
        return BlockWithHalo(outer, inner, local)

    def getNeighborId(self, block_id, axis, lower):
        c = self.blockCoordinates(block_id)
        c[axis] += -1 if lower else 1
        if c[axis] < 0 or c[axis] >= self.blocksPerAxis[axis]:
            return -1
        return int(sum(ci * s for ci, s in zip(c, self._strides)))

    def getBlockIdsOverlappingBoundingBox(self, roi_begin, roi_end):
        lo = [(max(b, rb) - rb) // s for b, rb, s in zip(roi_begin, self.roiBegin, self.blockShape)]
        hi = [(min(e, re) - 1 - rb) // s for e, re, rb, s in zip(roi_end, self.roiEnd, self.roiBegin,
                                                                  self.blockShape)]
        ranges = [range(l, h + 1) for l, h in zip(lo, hi)]
        ids = []
        for c in np.ndindex(*[len(r) for r in ranges]):
            cc = [r[i] for r, i in zip(ranges, c)]
            ids.append(int(sum(ci * s for ci, s in zip(cc, self._strides))))
        return np.array(sorted(ids), dtype='uint64')


def blocking(roiBegin, roiEnd, blockShape):
    return Blocking(roiBegin, roiEnd, blockShape)
