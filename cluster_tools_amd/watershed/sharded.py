"""Multi-GPU block sharding: one process per GPU, torch.distributed (RCCL on MI355X, gloo on CPU).

SURVEY.md §8(e).  Blocks are independent units (watershed.py:285-341), so a rank owns a
contiguous range of the C-order block list — z-slabs of the block grid — and processes it
without communication.  There are exactly two exchanges:

* the per-block label-count exchange that turns the block-local ids into compact global ids.
  The reference computes them with files: FindUniques writes per-job uniques, FindLabeling
  takes np.unique of their concatenation and numbers them consecutively
  (relabel/find_labeling.py:104-116; the same scan over per-block counts is
  thresholded_components/merge_offsets.py:106-122).  Watershed ids of block b are
  b * prod(block_shape) + local, so the sorted global uniques are the blocks' sorted uniques
  in block order, and the new id of the k-th nonzero unique of block b is
  1 + (number of nonzero uniques of the blocks before b) + k.  One all-gather of an int64 per
  block plus a prefix sum replaces the two file round trips.
* two-pass mode (two_pass_watershed.py:224-228): a pass-2 block reads the pass-1 labels of its
  halo, `initial_seeds = ds_out[input_bb]`.  Under z-slab sharding only the z-halo rows at a
  slab boundary belong to another rank; after pass 1 each rank sends its first / last
  halo[0] rows of labels to the neighbouring ranks (point-to-point over xGMI).

Single-process use needs no process group: the functions fall back to local computation.
With a process group (any world size, including 1) the exchanges go through it -- RCCL
(backend "nccl") on MI355X, gloo on CPU.  A gloo group also serves GPU tensors (ranks that
share a device, e.g. a 2-rank rehearsal on one GPU): they are staged through host memory.
"""
import numpy as np


def _dist():
    import torch.distributed as dist
    return dist if (dist.is_available() and dist.is_initialized()) else None


def comm_device(device=None):
    """The device the group's collectives take tensors on: `device` for RCCL, the host for gloo."""
    dist = _dist()
    if dist is not None and dist.get_backend() == 'gloo':
        return None
    return device


def all_reduce_max(value, device=None):
    """Max of a float over the ranks (the bench's max-over-ranks step time)."""
    import torch
    dist = _dist()
    if dist is None:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=comm_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_float(value, device=None):
    """Every rank's value, in rank order."""
    import torch
    dist = _dist()
    if dist is None:
        return [float(value)]
    t = torch.tensor([float(value)], dtype=torch.float64, device=comm_device(device))
    parts = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [float(p.item()) for p in parts]


def all_reduce_sum_int(value, device=None):
    import torch
    dist = _dist()
    if dist is None:
        return int(value)
    t = torch.tensor([int(value)], dtype=torch.int64, device=comm_device(device))
    dist.all_reduce(t)
    return int(t.item())


def shard_range(n_items, rank, world):
    """[begin, end) of the contiguous share of `rank` (sizes differ by at most one)."""
    return n_items * rank // world, n_items * (rank + 1) // world


def shard_blocks(block_list, rank, world):
    """The rank's contiguous share of a C-order block list (z-slabs of the block grid)."""
    b, e = shard_range(len(block_list), rank, world)
    return list(block_list[b:e])


def gather_counts(local_counts, device=None):
    """All-gather the per-block counts of every rank (ranks may hold different numbers of
    blocks).  Returns one int64 numpy array in rank order, i.e. global block order."""
    import torch
    dist = _dist()
    device = comm_device(device)
    local = torch.as_tensor(np.asarray(local_counts, dtype=np.int64), device=device)
    if dist is None:
        return local.cpu().numpy()
    world = dist.get_world_size()
    n = torch.tensor([local.numel()], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes)
    padded = torch.zeros(m, dtype=torch.int64, device=device)
    padded[:local.numel()] = local
    parts = [torch.zeros(m, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(parts, padded)
    return np.concatenate([p[:s].cpu().numpy() for p, s in zip(parts, sizes)])


def compact_offsets(all_counts):
    """Exclusive scan of the per-block nonzero-unique counts (global block order): block b's
    k-th nonzero id (k = 0, 1, ...) gets the new id offsets[b] + k + 1.  Also returns the new
    max id (relabel/find_labeling.py:108-116: 0 keeps 0, the others are numbered from 1)."""
    c = np.asarray(all_counts, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(c)[:-1]]) if len(c) else np.zeros(0, np.int64)
    return offs.astype(np.int64), int(c.sum())


def block_relabel_table(block_uniques, offset):
    """(old, new) of one block: its sorted uniques -> offset + 1 + rank (0 stays 0)."""
    u = np.asarray(block_uniques, dtype=np.uint64)
    nz = u[u != 0]
    new = np.arange(offset + 1, offset + 1 + len(nz), dtype=np.uint64)
    if len(nz) != len(u):
        return np.concatenate([[0], nz]).astype(np.uint64), np.concatenate([[0], new]).astype(np.uint64)
    return nz, new


def exchange_z_halos(vol, lo, hi):
    """Fill the z-halo rows of a rank's labels from its slab neighbours.

    `vol` is the rank's (lo + Z + hi, Y, X) tensor: rows [lo, lo + Z) are its own labels;
    rows [0, lo) receive the last lo own rows of rank - 1, rows [lo + Z, lo + Z + hi) the
    first hi own rows of rank + 1 (slabs are contiguous in rank order, so both neighbours'
    halos across a shared boundary have the same thickness).  Rows without a neighbouring
    rank are left as they are.  Point-to-point, one send and one receive per neighbour."""
    dist = _dist()
    if dist is None or dist.get_world_size() == 1:
        return vol
    rank, world = dist.get_rank(), dist.get_world_size()
    Z = vol.shape[0] - lo - hi
    host = comm_device(vol.device) is None and vol.device.type != 'cpu'  # gloo: through the host

    def out(t):
        return t.cpu() if host else t.contiguous()

    def buf(n):
        shape = (n,) + tuple(vol.shape[1:])
        return vol.new_empty(shape, device='cpu') if host else vol.new_empty(shape)
    ops, recv_lo, recv_hi = [], None, None
    if rank > 0 and lo:
        ops.append(dist.P2POp(dist.isend, out(vol[lo:2 * lo]), rank - 1))
        recv_lo = buf(lo)
        ops.append(dist.P2POp(dist.irecv, recv_lo, rank - 1))
    if rank + 1 < world and hi:
        ops.append(dist.P2POp(dist.isend, out(vol[lo + Z - hi:lo + Z]), rank + 1))
        recv_hi = buf(hi)
        ops.append(dist.P2POp(dist.irecv, recv_hi, rank + 1))
    if ops:
        for r in dist.batch_isend_irecv(ops):
            r.wait()
    if recv_lo is not None:
        vol[:lo] = recv_lo
    if recv_hi is not None:
        vol[lo + Z:] = recv_hi
    return vol


def exchange_z_halo_boxes(vol, lo, hi, send_lo, send_hi, recv_lo, recv_hi):
    """exchange_z_halos restricted to (y0, y1, x0, x1) boxes of the halo rows: the rank sends
    its first lo own rows inside the `send_lo` boxes to rank - 1 and its last hi own rows inside
    `send_hi` to rank + 1, and fills its lower / upper halo rows inside `recv_lo` / `recv_hi`
    (the boxes the neighbour sends, in the same order).  Every rank derives the boxes from the
    same schedule (pass2_rank_schedule), so sends and receives pair up; an empty list skips that
    transfer on both sides.  Point-to-point, concatenated boxes per neighbour."""
    dist = _dist()
    if dist is None or dist.get_world_size() == 1:
        return vol
    rank, world = dist.get_rank(), dist.get_world_size()
    Z = vol.shape[0] - lo - hi
    host = comm_device(vol.device) is None and vol.device.type != 'cpu'

    def pack(z0, z1, boxes):
        parts = [vol[z0:z1, y0:y1, x0:x1].reshape(-1) for y0, y1, x0, x1 in boxes]
        t = parts[0].new_empty(0) if not parts else (parts[0] if len(parts) == 1 else torch.cat(parts))
        return t.cpu() if host else t.contiguous()

    def nvals(n, boxes):
        return n * sum((y1 - y0) * (x1 - x0) for y0, y1, x0, x1 in boxes)

    def unpack(buf, z0, z1, boxes):
        buf = buf.to(vol.device) if host else buf
        o = 0
        for y0, y1, x0, x1 in boxes:
            m = (z1 - z0) * (y1 - y0) * (x1 - x0)
            vol[z0:z1, y0:y1, x0:x1] = buf[o:o + m].view(z1 - z0, y1 - y0, x1 - x0)
            o += m
    import torch
    ops, rl, rh = [], None, None
    dev = 'cpu' if host else vol.device
    if rank > 0 and lo:
        if send_lo:
            ops.append(dist.P2POp(dist.isend, pack(lo, 2 * lo, send_lo), rank - 1))
        if recv_lo:
            rl = torch.empty(nvals(lo, recv_lo), dtype=vol.dtype, device=dev)
            ops.append(dist.P2POp(dist.irecv, rl, rank - 1))
    if rank + 1 < world and hi:
        if send_hi:
            ops.append(dist.P2POp(dist.isend, pack(lo + Z - hi, lo + Z, send_hi), rank + 1))
        if recv_hi:
            rh = torch.empty(nvals(hi, recv_hi), dtype=vol.dtype, device=dev)
            ops.append(dist.P2POp(dist.irecv, rh, rank + 1))
    if ops:
        for r in dist.batch_isend_irecv(ops):
            r.wait()
    if rl is not None:
        unpack(rl, 0, lo, recv_lo)
    if rh is not None:
        unpack(rh, lo + Z, lo + Z + hi, recv_hi)
    return vol


def all_gather_ints(values, device=None):
    """Every rank's list of ints, concatenated in rank order."""
    return [int(v) for v in gather_counts(values, device=device)]


def pass2_rank_schedule(p2_blocks, slabs, hz, boxes=False):
    """The two-pass watershed's sequential schedule over z-slab ranks.

    p2_blocks: the pass-2 blocks of the whole job that write something, in the sequential list
    order (two_pass_watershed.py:296-299), as (owner rank, input_bb, output_bb) with global
    bounding boxes; slabs: [(z0, z1)] per rank; hz: the z halo.  Returns (levels, exchange):
    levels[k] = the level of block k (watershed.pass2_levels over the global list, so a block
    reads after every earlier block it overlaps wrote, on whichever rank that one ran);
    exchange[l] = whether the z-halo rows must be exchanged before level l: before level 0
    (the pass-1 labels) and after every level with a block whose output rows lie within hz of
    its slab's boundary to a neighbouring rank (another rank's halo reads them).  Every rank
    computes the same schedule, so all of them exchange at the same levels.
    With boxes=True also returns, per level l >= 1, {(owner, 'lo' | 'hi'): [(y0, y1, x0, x1)]}:
    the (y, x) footprints of the level-(l - 1) blocks each rank must send down ('lo', to
    owner - 1) or up ('hi', to owner + 1) -- only those rows changed since the last exchange."""
    from cluster_tools_amd.watershed.watershed import pass2_levels
    levels = pass2_levels([(ib, ob) for _, ib, ob in p2_blocks])
    n_levels = max(levels) + 1 if levels else 0
    exchange = [False] * n_levels
    if n_levels:
        exchange[0] = True
    world = len(slabs)
    bx = [dict() for _ in range(n_levels)]
    for (r, _, ob), lv in zip(p2_blocks, levels):
        z0, z1 = slabs[r]
        b0, b1 = ob[0].start, ob[0].stop
        dn = r > 0 and b0 < z0 + hz
        up = r + 1 < world and b1 > z1 - hz
        if (dn or up) and lv + 1 < n_levels:
            exchange[lv + 1] = True
            fp = (ob[1].start, ob[1].stop, ob[2].start, ob[2].stop)
            if dn:
                bx[lv + 1].setdefault((r, 'lo'), []).append(fp)
            if up:
                bx[lv + 1].setdefault((r, 'hi'), []).append(fp)
    if boxes:
        return levels, exchange, bx
    return levels, exchange
