"""Development check: GPU (libctws) vs CPU oracle, stage by stage, on synthetic blocks."""
import sys
import time
import numpy as np

sys.path.insert(0, '.')
from cluster_tools_amd import ctws
from cluster_tools_amd.synthetic import boundary_map, ellipsoid_mask
from cluster_tools_amd.metrics import vi_scores, rand_scores
from oracle import oracle as O


def run_case(h, name, config, x, mask=None, inner=None, crop=False, block_id=3, block_shape=(64, 256, 256)):
    shape = x.shape[-3:]
    b = dict(input=x, mask=mask, block_id=block_id, crop_relabel=crop)
    if inner is not None:
        b['inner_begin'], b['inner_shape'] = inner
    t = time.time()
    ref = O.ws_blocks(config, block_shape, [b], with_stages=True)[0]
    tcpu = time.time() - t
    stages = {}
    for stop, names in ((1, ('fin', 'dt', 'seedmap', 'hmap', 'labels')), (3, ('labels',))):
        h.debug_set_stop(stop)
        h.ws_blocks(config, block_shape, [dict(b)])
        for nm in names:
            stages[(stop, nm)] = h.debug_read(nm, 0, shape)
    h.debug_set_stop(0)
    t = time.time()
    res = h.ws_blocks(config, block_shape, [dict(b)])[0]
    tgpu = time.time() - t
    tm = h.timings()
    out = res['output']
    print("== %s  shape %s  cpu %.2fs  gpu %.3fs  status %d/%d" % (name, shape, tcpu, tgpu, res['status'], ref['status']))
    print("   timings", {k: round(v, 3) for k, v in tm.items()})
    if ref['status'] != 0:
        print("   output equal:", np.array_equal(out, ref['output']))
        return
    fin = stages[(1, 'fin')]
    print("   fin exact:", np.array_equal(fin, ref['input']), " dt exact:", np.array_equal(stages[(1, 'dt')], ref['dt']),
          " dt maxdiff", float(np.abs(stages[(1, 'dt')] - ref['dt']).max()))
    nd = 2 if config.get('apply_ws_2d', True) else 3
    dt = ref['dt']
    if nd == 3:
        seeds_ref = O.make_seeds(dt, config)
        hm_ref = O.make_hmap(ref['input'], dt, config)
        sm_ref = O.gaussian_smoothing(dt, config.get('sigma_seeds', 2.)) if config.get('sigma_seeds', 2.) else dt
    else:
        seeds_ref = np.zeros(shape, np.uint32); hm_ref = np.zeros(shape, np.float32); sm_ref = np.zeros(shape, np.float32)
        nseen = 0
        for z in range(shape[0]):
            s = O.make_seeds(dt[z], config)
            s[s > 0] += nseen
            nseen = max(nseen, int(s.max()))
            seeds_ref[z] = s
            hm_ref[z] = O.make_hmap(ref['input'][z], dt[z], config)
            sg = config.get('sigma_seeds', 2.)
            sm_ref[z] = O.gaussian_smoothing(dt[z], sg) if sg else dt[z]
    sm = stages[(1, 'seedmap')]
    print("   seedmap exact:", np.array_equal(sm, sm_ref), " maxrel", float((np.abs(sm - sm_ref) / np.maximum(np.abs(sm_ref), 1e-6)).max()))
    hm = stages[(1, 'hmap')]
    print("   hmap exact:", np.array_equal(hm, hm_ref), " maxdiff", float(np.abs(hm - hm_ref).max()))
    seeds = stages[(1, 'labels')] & 0x7FFFFFFF
    print("   seeds exact:", np.array_equal(seeds, seeds_ref), " n", int(seeds.max()), int(seeds_ref.max()),
          " mismatched voxels", int((seeds != seeds_ref).sum()))
    ws = stages[(3, 'labels')]
    ign = [0] if mask is not None else None
    print("   ws  VI(split,merge)", vi_scores(ws, ref['ws'], ign), " ARE", rand_scores(ws, ref['ws'], ign)[0],
          " equal frac", float((ws == ref['ws']).mean()))
    print("   out VI", vi_scores(out, ref['output'], ign), " ARE", rand_scores(out, ref['output'], ign)[0],
          " exact", np.array_equal(out, ref['output']), " equal frac", float((out == ref['output']).mean()))


def main():
    h = ctws.Handle(0)
    x3 = boundary_map((32, 96, 96), seed=1)
    run_case(h, '3d default', dict(apply_dt_2d=False, apply_ws_2d=False), x3)
    run_case(h, '2d default', {}, x3)
    run_case(h, '2d test cfg', dict(threshold=.25, sigma_weights=0., halo=[0, 32, 32]), x3,
             inner=((0, 16, 16), (32, 64, 64)), crop=True)
    run_case(h, '3d aniso', dict(apply_dt_2d=False, apply_ws_2d=False, sigma_seeds=(.5, 2., 2.), sigma_weights=(.5, 2., 2.)), x3,
             inner=((2, 16, 16), (28, 64, 64)), crop=True)
    run_case(h, '3d pitch', dict(apply_dt_2d=False, apply_ws_2d=False, pixel_pitch=(10, 1, 1)), x3)
    m = ellipsoid_mask(x3.shape)
    run_case(h, '3d mask', dict(apply_dt_2d=False, apply_ws_2d=False), x3, mask=m)
    run_case(h, '2d mask', {}, x3, mask=m)
    x4 = np.stack([boundary_map((32, 96, 96), seed=s) for s in (4, 5, 6)])
    run_case(h, '4d mean', dict(apply_dt_2d=False, apply_ws_2d=False), x4)
    xb = boundary_map((64, 256, 256), seed=0)
    run_case(h, '3d big', dict(apply_dt_2d=False, apply_ws_2d=False), xb)


if __name__ == '__main__':
    main()
