"""Pipeline stage of every ctws:: kernel dispatch, from the dispatch order of one library stream
(bench.py --streams 1): a state machine over the kernel names that mirrors run_batch's stage marks
(ctws_api.cpp mark(...)).  Shared by pmc_traffic.py (HBM bytes per stage) and
roofline_from_trace.py (kernel time per stage), so that traffic and time cover the same
dispatches.

Stages: prep_edt_x, edt_yz, smooth_seeds, hmap, seeds, flood, size_filter, crop_cc, output.
The flood is every dispatch from a batch's k_descent_tile (or, without the descent, its first
flood kernel) up to the size filter's first kernel; the size filter's regrow (k_regrow_init, its
frontier launches and its fixpoint check) belongs to size_filter."""


def short(name):
    return name.split('(')[0].replace('void ', '').replace('ctws::', '').strip()


def base(name):
    return short(name).split('<')[0]


GAUSS = ('k_gauss_yx', 'k_gauss_col_r', 'k_gauss_row_r', 'k_gauss_col', 'k_gauss_row', 'k_hmap')
FLOOD_START = ('k_descent_tile', 'k_flood_packed', 'k_flood')
SIZE_FILTER_START = ('k_hist_zero', 'k_size_filter')
CROP = ('k_slice_max', 'k_slice_offsets', 'k_finalize_ws', 'k_p2_check', 'k_slice_inmask', 'k_flatten_tile_roots')
OUTPUT = ('k_output', 'k_output_crop', 'k_count_ids', 'k_p2_output', 'k_fs_output')


def classify(names):
    """names: kernel names of one stream's dispatches in launch order -> list of stage names
    (None for non-library kernels)."""
    out = []
    state = None
    gauss_seen = 0       # Gaussian-family dispatches of the current batch so far
    gauss_total = 0      # ... and in the whole batch (precomputed per batch below)
    # Gaussian dispatches per batch, to split the seed-map and hmap smoothing
    batch_gauss = []
    cnt = None
    for n in names:
        b = base(n) if 'ctws::' in n else None
        if b in ('k_input_minmax', 'k_input_minmax_t'):
            if cnt is not None:
                batch_gauss.append(cnt)
            cnt = 0
        elif b in GAUSS and cnt is not None:
            cnt += 1
    if cnt is not None:
        batch_gauss.append(cnt)
    bi = -1
    for n in names:
        if 'ctws::' not in n:
            out.append(None)
            continue
        b, s = base(n), short(n)
        if b in ('k_input_minmax', 'k_input_minmax_t'):
            state = 'prep_edt_x'
            bi += 1
            gauss_seen = 0
            gauss_total = batch_gauss[bi] if 0 <= bi < len(batch_gauss) else 0
        elif b.startswith('k_edt') or b in ('k_dt_slice_stats', 'k_p2_zero_dt'):
            if state in (None, 'prep_edt_x', 'edt_yz'):
                state = 'edt_yz'
        elif b in GAUSS:
            gauss_seen += 1
            # k_hmap (no weights smoothing) is the hmap; otherwise the second half of the batch's
            # Gaussian dispatches (seed map first, then hmap; equal pass counts in the default
            # configs: 2-D 1 + 1 fused y/x tiles, 3-D 3 + 3 axis passes)
            if b == 'k_hmap' or gauss_seen > (gauss_total + 1) // 2:
                state = 'hmap'
            else:
                state = 'smooth_seeds'
        elif b == 'k_localmax':
            state = 'seeds'
        elif b in FLOOD_START and state in ('seeds', 'hmap', 'smooth_seeds', 'edt_yz', 'prep_edt_x'):
            state = 'flood'
        elif b in SIZE_FILTER_START and state == 'flood':
            state = 'size_filter'
        elif (b in CROP or (b in ('k_tile_cc', 'k_tile_merge') and s.endswith(', 2>'))) and \
                state in ('flood', 'size_filter'):
            state = 'crop_cc'
        elif b in OUTPUT:
            state = 'output'
        out.append(state)
    return out
