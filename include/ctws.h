/*
 * ctws.h — C-ABI of libctws.so, the MI355X (gfx950) blockwise DT-watershed.
 *
 * This is the drop-in boundary for the hot path of cluster_tools' watershed task.
 * Every entry point is plain C: pointers, sizes, POD structs.  No torch / HIP types.
 *
 * Reference interfaces each entry point replaces (paths relative to the reference repo):
 *
 *   ctws_ws_blocks / ctws_ws_blocks_device
 *       the per-job block loop `for block_id in block_list: _ws_block(...)`
 *       cluster_tools/watershed/watershed.py:380-381, i.e. `_ws_block` (:285-341) with
 *       `_read_data` (:267-282), `_apply_dt` (:139-160), `_make_seeds` (:179-207),
 *       `_make_hmap` (:163-169), `_apply_watershed` (:211-249) and the halo crop /
 *       labelVolumeWithBackground / id offset (:326-341);
 *       and, with cfg.pass_id == 1, `_ws_pass2`
 *       cluster_tools/watershed/two_pass_watershed.py:210-255 (+ :122-207).
 *       The caller does the dataset I/O (ds_in[input_bb], ds_out[output_bb] = ...) and the
 *       "processed block" log lines, exactly as the reference job entry does.
 *
 *   ctws_ws_from_seeds / ctws_ws_from_seeds_device
 *       the WatershedFromSeeds job loop (watershed/watershed_from_seeds.py:236-249 over
 *       `_ws_block` / `_ws_block_masked`, :143-199).
 *
 *   ctws_eval_begin / ctws_eval_add / ctws_eval_end
 *       EvaluationWorkflow's overlaps + Measures (evaluation/evaluation_workflow.py:53-77,
 *       evaluation/measures.py:80-164, utils/validation_utils.py:60-76, 178-198).
 *
 *   ctws_threshold_components / ctws_ufd_find
 *       ThresholdedComponentsWorkflow: BlockComponents' per-block `_cc_block[_with_mask]`
 *       (thresholded_components/block_components.py:143-230: normalize, threshold,
 *       skimage.morphology.label) and MergeAssignments' nifty boost_ufd merge + find
 *       (thresholded_components/merge_assignments.py:125-130).
 *
 *   ctws_open / ctws_close / ctws_last_error
 *       process-level setup; the reference has none (vigra is stateless).  One handle per
 *       (process, GPU), as LocalTask runs one process per job (cluster_tasks.py:507-529).
 *
 *   (multi-GPU) the library holds no communicator: the per-block label counts it returns
 *       (ctws_block.n_ids) are all-gathered and exclusively scanned by the host over
 *       torch.distributed (RCCL, cluster_tools_amd/watershed/sharded.py), replacing the
 *       FindUniques -> FindLabeling file exchange (relabel/find_labeling.py:104-116,
 *       thresholded_components/merge_offsets.py:111-119).
 *
 * Conventions
 *   - all arrays are C-contiguous numpy-order arrays (axis 0 = z slowest, axis 2 = x fastest)
 *   - the caller owns every buffer it passes; no pointer is retained after return
 *   - return value 0 = ok, negative = error; the message is in ctws_last_error(h)
 *   - calls on one handle are serialized (not re-entrant); use one handle per thread
 */
#ifndef CTWS_H
#define CTWS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CTWS_ABI_VERSION 2

/* error codes */
#define CTWS_OK            0
#define CTWS_EINVAL       -1  /* bad argument                                    */
#define CTWS_EHIP         -2  /* HIP runtime error                               */
#define CTWS_ENOMEM       -3  /* device allocation failed                        */
#define CTWS_ECOMM        -4  /* RCCL error                                      */
#define CTWS_EUNSUPPORTED -5  /* configuration the kernels do not implement      */

/* input dtypes (ds_in dtype; the reference casts to float32 in normalize) */
#define CTWS_U8  1
#define CTWS_U16 2
#define CTWS_F32 3
#define CTWS_F64 4
/* further dtypes of ctws_threshold_components_ex (BlockComponents thresholds the raw dataset) */
#define CTWS_I8  5
#define CTWS_I16 6
#define CTWS_I32 7
#define CTWS_U32 8
#define CTWS_I64 9
#define CTWS_U64 10

/* agglomerate_channels */
#define CTWS_AGG_MEAN 0
#define CTWS_AGG_MAX  1
#define CTWS_AGG_MIN  2

/* per-block status written by ctws_ws_blocks */
#define CTWS_BLOCK_WRITTEN      0  /* output holds the block's uint64 labels           */
#define CTWS_BLOCK_SKIPPED_MASK 1  /* inner mask empty: nothing written (:295-297)     */
#define CTWS_BLOCK_EMPTY        2  /* nothing above threshold: constant offset written */
#define CTWS_BLOCK_EMPTY_PASS2  3  /* pass 2, nothing above threshold: nothing written */
#define CTWS_BLOCK_FAILED       4  /* the block cannot be finished: nothing written;    */
                                   /* the reason is in ctws_last_error (the reference   */
                                   /* job would raise at this block)                    */

/*
 * Task configuration.  Mirrors the watershed task config keys
 * (watershed.py:50-60, two_pass_watershed.py:39-49) with the inline defaults the job
 * code applies (config.get(k, default)).
 */
typedef struct ctws_cfg {
    double  threshold;               /* 'threshold' (compared in float32)                  */
    double  alpha;                   /* 'alpha'                                            */
    double  sigma_seeds[3];          /* 'sigma_seeds': scalar in [0] or per-axis list      */
    int32_t sigma_seeds_is_list;     /*   1 if the config held a list/tuple                */
    double  sigma_weights[3];        /* 'sigma_weights'                                    */
    int32_t sigma_weights_is_list;
    int32_t size_filter;             /* 'size_filter'                                      */
    int32_t apply_dt_2d;             /* 'apply_dt_2d'                                      */
    int32_t apply_ws_2d;             /* 'apply_ws_2d'                                      */
    int32_t has_pixel_pitch;         /* 'pixel_pitch' is not None                          */
    double  pixel_pitch[3];
    int32_t invert_inputs;           /* 'invert_inputs'                                    */
    int32_t channel_begin;           /* 'channel_begin'                                    */
    int32_t channel_end;             /* 'channel_end', < 0 means None                      */
    int32_t agglomerate_channels;    /* CTWS_AGG_*                                         */
    int32_t non_maximum_suppression; /* must be 0: nifty NMS is not available (:20-23)     */
    int32_t pass_id;                 /* 0 = _ws_block, 1 = _ws_pass2                       */
    int64_t block_shape[3];          /* global block shape: offset = id * prod(shape)      */
} ctws_cfg;

/*
 * One block.  `input` holds the OUTER block (block + halo, clipped to the volume) as
 * ds_in[input_bb] would return it; `output` receives ws[inner_bb] as uint64.
 */
typedef struct ctws_block {
    const void*     input;           /* [C][Z][Y][X] (n_channels > 0) or [Z][Y][X]         */
    int32_t         input_dtype;     /* CTWS_U8 / U16 / F32 / F64                          */
    int32_t         n_channels;      /* 0 for a 3-D dataset                                */
    int64_t         outer_shape[3];  /* Z, Y, X of the outer block                         */
    const uint8_t*  mask;            /* outer-shaped, nonzero = in mask; NULL = no mask    */
    int64_t         inner_begin[3];  /* inner block, local to the outer block              */
    int64_t         inner_shape[3];
    int32_t         crop_relabel;    /* 1 iff output_bb != input_bb (:327)                 */
    int32_t         _pad0;
    int64_t         block_id;        /* id offset = block_id * prod(cfg.block_shape)       */
    const uint64_t* initial_seeds;   /* pass 2: ds_out[input_bb], outer-shaped; else NULL  */
    uint64_t*       output;          /* inner-shaped uint64                                */
    uint64_t        max_label;       /* out: largest local label before the id offset      */
    int32_t         status;          /* out: CTWS_BLOCK_*                                  */
    int32_t         n_ids;           /* out: distinct nonzero output ids of the block (pass */
                                     /* 0; -1 in pass 2): the per-block count of the       */
                                     /* compact-id exclusive scan (find_labeling.py:104)   */
} ctws_block;

typedef struct ctws_handle ctws_handle;

/* version of this header the library was built against */
int ctws_abi_version(void);

/* open the library on HIP device `device` (index within HIP_VISIBLE_DEVICES) */
int ctws_open(int device, ctws_handle** out);
void ctws_close(ctws_handle* h);
const char* ctws_last_error(const ctws_handle* h);

/*
 * Run the watershed of `n_blocks` blocks.  input/mask/initial_seeds/output are HOST
 * pointers.  The blocks run in device-memory-sized batches; each batch's inputs are packed
 * (multi-threaded memcpy) into one of two pinned host buffers and uploaded on a copy stream
 * while the previous batch computes, and its outputs are downloaded on a second copy stream
 * and unpacked while the next batch computes.  The pinned and device staging buffers are kept
 * by the handle (grow-only) for later calls.
 */
int ctws_ws_blocks(ctws_handle* h, const ctws_cfg* cfg, ctws_block* blocks, int n_blocks);

/*
 * Same, but input/mask/initial_seeds/output are DEVICE pointers on the handle's GPU
 * (e.g. torch tensors' data_ptr()).  Work is enqueued on the handle's stream and the
 * call returns after the stream has drained.
 */
int ctws_ws_blocks_device(ctws_handle* h, const ctws_cfg* cfg, ctws_block* blocks, int n_blocks);

/*
 * WatershedFromSeeds (watershed/watershed_from_seeds.py:143-199, `_ws_block` and
 * `_ws_block_masked`): per block, input = normalize(ds_in[bb]) (4-D: channel range +
 * agglomeration; no invert), masked voxels -> 1, seeds = `initial_seeds` (= ds_seeds[bb],
 * uint64, the block's shape), ws = watershedsNew(input, seeds) (3-D, direct nbhd) + the
 * size filter (cfg.size_filter), ws[~mask] = 0 -> `output` (uint64).  Blocks have no halo:
 * inner_begin = 0, inner_shape = outer_shape.  Only threshold-independent keys of `cfg` are
 * read (size_filter, channel_begin/end, agglomerate_channels).  A block whose seeds hold an
 * id >= 2^32 - 1 gets CTWS_BLOCK_FAILED (the reference's "Overflow detected" assert); a block
 * with an empty mask CTWS_BLOCK_SKIPPED_MASK (nothing written).  max_label = largest output id.
 */
int ctws_ws_from_seeds(ctws_handle* h, const ctws_cfg* cfg, ctws_block* blocks, int n_blocks);
int ctws_ws_from_seeds_device(ctws_handle* h, const ctws_cfg* cfg, ctws_block* blocks, int n_blocks);

/*
 * Evaluation (evaluation/measures.py:80-164 with utils/validation_utils.py:60-76, 178-198):
 * the seg x gt contingency table built in HBM (hash tables of gt ids, seg ids and id pairs
 * with voxel counts), accumulated over any number of ctws_eval_add calls (blockwise), then
 * reduced.  cap_labels / cap_pairs bound the distinct ids per side / distinct pairs; a full
 * table makes ctws_eval_end return CTWS_EUNSUPPORTED (retry with larger capacities).
 * ignore_gt_zero drops voxels whose gt label is 0 (EvaluationWorkflow(ignore_label=True),
 * evaluation_workflow.py:53,60).  scores = {vi_split, vi_merge, adapted_rand_error,
 * rand_index} (log2), exactly the keys measures() writes.
 */
int ctws_eval_begin(ctws_handle* h, int64_t cap_labels, int64_t cap_pairs);
int ctws_eval_add(ctws_handle* h, const uint64_t* seg, const uint64_t* gt, int64_t n, int on_device,
                  int ignore_gt_zero);
int ctws_eval_end(ctws_handle* h, double* scores /* [4] */, int64_t* n_points);

/*
 * Stage timings of the last ctws_ws_blocks* call, measured with HIP events on the
 * handle's stream (milliseconds).  names[i] is a static string.  Returns the count.
 */
int ctws_last_timings(const ctws_handle* h, const char** names, float* ms, int max_entries);

/*
 * RelabelWorkflow (relabel/find_uniques.py:93-159, find_labeling.py:84-126,
 * write/write.py:153-226) on the GPU.  on_device = 1: labels/out/keys/values are device
 * pointers on the handle's GPU; 0: host pointers (staged through HBM).
 *
 * ctws_unique_u64: the sorted unique values of labels[0..n) (np.unique) into out[0..cap);
 *   *n_unique = their number (also when cap is too small: then CTWS_EINVAL, retry with a
 *   larger buffer).  Any value range: a bitmap over the range when it is dense enough
 *   (watershed ids), else a radix sort.  Fewer than 2^31 labels per call.
 * ctws_unique_counts_u64: np.unique(labels, return_counts=True) (find_uniques.py:104-106):
 *   sorted uniques into out, their voxel counts into counts (both cap entries).
 * ctws_set_table_u64: upload an assignment table (host keys ascending, values) and keep it
 *   resident on the handle (one upload per Write job instead of one per block).
 * ctws_lookup_u64: labels[i] <- values[j] where keys[j] == labels[i] (keys ascending;
 *   nifty.tools.takeDict); labels absent from the table are left unchanged and counted in
 *   *n_missing (takeDict would raise: the caller raises).  keys == values == NULL: use the
 *   resident table; host keys/values (on_device = 0) become the resident table.
 */
int ctws_set_table_u64(ctws_handle* h, const uint64_t* keys, const uint64_t* values, int64_t n_table);
int ctws_unique_u64(ctws_handle* h, const uint64_t* labels, int64_t n, int on_device, uint64_t* out, int64_t cap,
                    int64_t* n_unique);
int ctws_unique_counts_u64(ctws_handle* h, const uint64_t* labels, int64_t n, int on_device, uint64_t* out,
                           uint64_t* counts, int64_t cap, int64_t* n_unique);
int ctws_lookup_u64(ctws_handle* h, uint64_t* labels, int64_t n, int on_device, const uint64_t* keys,
                    const uint64_t* values, int64_t n_table, int64_t* n_missing);

/*
 * ThresholdedComponentsWorkflow, BlockComponents (thresholded_components/block_components.py:
 * 143-230: `_cc_block` / `_cc_block_with_mask`, threshold + skimage.morphology.label) on the GPU.
 *
 * ctws_threshold_components: input = one float32 block (nz, ny, nx), C order; mask = uint8
 *   (nonzero = in mask) or NULL; normalize = 1 applies vu.normalize first (the unmasked,
 *   single-channel case); mode 0 'greater', 1 'less', 2 'equal' against threshold (compared as
 *   float32).  out (uint64, same shape) <- the 26-connected components of the members numbered
 *   1.. in order of first appearance in a C-order scan (skimage's numbering), 0 elsewhere;
 *   *n_labels = their number.  A block without members leaves out unwritten and *n_labels = 0
 *   (the reference returns 0 and writes nothing).  on_device: 1 device pointers, 0 host.
 *   Blocks of fewer than 2^32 - 1 voxels; a device input is 16-byte aligned when normalize = 1
 *   (CTWS_EINVAL otherwise; torch / hipMalloc allocations are).
 */
int ctws_threshold_components(ctws_handle* h, const float* input, const uint8_t* mask, int64_t nz, int64_t ny,
                              int64_t nx, int on_device, int mode, double threshold, int normalize, uint64_t* out,
                              int64_t* n_labels);
/*
 * ctws_threshold_components_ex: the same for any dtype of the dataset and with the Gaussian
 * prefilter (block_components.py:150-171 `_cc_block`, :198-222 `_cc_block_with_mask`):
 *   x = input (dtype: CTWS_U8 .. CTWS_U64); if normalize: x = vu.normalize(x) (float32);
 *   if sigma > 0: x = vu.normalize(gaussianSmoothing(float32(x), sigma)) (vigra: radius
 *   int(3 sigma + 0.5), reflect border, double accumulation, float32 between the axes);
 *   members = x `mode` threshold.  The comparison is numpy's for `x > python float`: float32
 *   against the threshold rounded to float32 when x is float32 (normalized, smoothed or a
 *   float32 dataset), float64 otherwise (float64 and integer datasets, NEP 50).  The caller
 *   passes normalize = 1 for an unmasked single-channel block (`_cc_block` normalizes the raw
 *   block) and for a masked block with sigma > 0 (`_cc_block_with_mask` normalizes before the
 *   filter).  A line shorter than radius + 1 along any axis is refused as vigra refuses it.
 */
int ctws_threshold_components_ex(ctws_handle* h, const void* input, int dtype, const uint8_t* mask, int64_t nz,
                                 int64_t ny, int64_t nx, int on_device, int mode, double threshold, int normalize,
                                 double sigma, uint64_t* out, int64_t* n_labels);
/*
 * MergeAssignments (thresholded_components/merge_assignments.py:125-130): out[i] = the
 * representative of label i after merging the (a, b) rows of pairs (n_pairs x 2, C order) into
 * nifty's boost_ufd(n) in row order -- boost::disjoint_sets union by rank (equal ranks: the first
 * root goes under the second).  Host code, no handle; CTWS_EINVAL for a label >= n.
 */
int ctws_ufd_find(int64_t n, const uint64_t* pairs, int64_t n_pairs, uint64_t* out);

/*
 * Test hooks (used by the parity tests, not by the task code): stop the pipeline after a
 * stage and read back one block's outer-shaped workspace array of the last batch.
 *   arrays: "fin" (float32 normalized input), "dt" (float32), "seedmap" (float32 smoothed
 *           dt), "hmap" (float32), "labels" (uint32; bit 31 = seed), "cls" (uint8)
 */
#define CTWS_STOP_NONE  0
#define CTWS_STOP_SEEDS 1  /* after seed labelling (labels = seeds)            */
#define CTWS_STOP_FLOOD 2  /* after the first flood (labels = watershed)        */
#define CTWS_STOP_WS    3  /* after the size filter + 2-D offsets + masking     */
int ctws_debug_set_stop(ctws_handle* h, int stage);
int ctws_debug_read(ctws_handle* h, const char* array, int block, void* dst, int64_t nbytes);
/* the EDT's correctly rounded sqrt of integers n0 .. n0 + count - 1 (< 2^24) into host dst */
int ctws_debug_sqrt_int(ctws_handle* h, uint32_t n0, uint32_t count, float* dst);

#ifdef __cplusplus
}
#endif

#endif /* CTWS_H */
