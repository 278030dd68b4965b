/*
 * rfrt.h -- C ABI of librfrt.so, the MI355X-native replacement for the Warp hot path of
 * rmenon1008/rf_ray_tracing_warp.  Plain pointers and sizes only; every device pointer is
 * caller-owned (e.g. a PyTorch tensor's data_ptr()) and every launch is asynchronous on the
 * caller's hipStream_t (pass NULL for the default stream).
 *
 * Error convention: functions return RT_OK (0) or a negative code; rt_last_error() gives the
 * message of the last failure on the calling thread.  Nothing throws across the ABI.
 * Threading: mesh create/destroy are not thread-safe for the same handle; launches are
 * reentrant.  Reference paths below are relative to the reference repository root.
 */
#ifndef RFRT_H
#define RFRT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RFRT_VERSION 1

#define RT_OK 0
#define RT_EINVAL (-1) /* bad argument: Warp raises a Python exception at launch (tracer.py:75) */
#define RT_EHIP (-2)   /* HIP runtime error */

/* rt_cir flags: NumPy 2 / NEP 50 promotes tracer.py:115 to float64 when light_speed_mps or
 * sample_rate_hz is a NumPy float64 scalar instead of a Python float. */
#define RT_CIR_C_F64 1
#define RT_CIR_FS_F64 2

typedef struct rt_mesh rt_mesh;

const char* rt_last_error(void);
int rt_version(void);

/* Replaces wp.Mesh(points=wp.array(vertices, vec3), velocities=None, indices=wp.array(faces.flatten(),
 * int32)) -- tracer.py:22-24 (environment) and tracer.py:28-30 (receiver sphere).
 * vertices: host float32 (nv,3); faces: host int32 (nf,3).  Builds the device tables (and a BVH
 * for large meshes) on `device`; the library owns the handle. */
int rt_mesh_create(int device, const float* vertices, int64_t nv, const int32_t* faces, int64_t nf, rt_mesh** out);
/* rt_mesh_create with builder flags: 0 = host binned-SAH BVH (default, best trees),
 * RT_MESH_BVH_GPU = device LBVH over Morton codes (milliseconds for millions of
 * faces; falls back to the host build if its tree is deeper than the traversal stack).  Meshes
 * of <= 192 faces are traced by brute force and have no BVH either way; results never depend on
 * the tree (closest hit = lexicographic (t, face) minimum). */
#define RT_MESH_BVH_GPU 1
int rt_mesh_create_ex(int device, const float* vertices, int64_t nv, const int32_t* faces, int64_t nf, int flags,
                      rt_mesh** out);
/* Replaces the wp.Mesh destructor (freed on Python GC in the reference). */
int rt_mesh_destroy(rt_mesh* mesh);
/* nf, bounds6 = (lo xyz, hi xyz), sphere4 = conservative bounding sphere (centre, radius). Any may be NULL. */
int rt_mesh_info(const rt_mesh* mesh, int64_t* nf, float* bounds6, float* sphere4);
/* BVH statistics (all 0 for meshes of <= 192 faces, which are traced by brute force):
 * info4 = (nodes, leaves, max internal-node depth, max faces in a leaf).  No reference
 * counterpart: Warp's wp.Mesh BVH (tracer.py:24) is internal. */
int rt_bvh_info(const rt_mesh* mesh, int64_t* info4);

/* rt_trace keeps, per process, up to 8 direction-sorted ray orders (per device, ray_offset and n:
 * 4 bytes per ray) and up to 8 chunk schedules (per device, burst, meshes and TX; a mesh's are
 * dropped by rt_mesh_destroy).  This frees all of them (the next rt_trace recomputes what it needs;
 * no result depends on them).  Synchronises the devices it frees memory on.  No reference
 * counterpart (Warp keeps no such state). */
int rt_release_caches(void);

/* Replaces wp.launch(kernel.trace_paths_kernel, dim=(n,1,1), inputs=[env.id, tx_pos, rx.id,
 * max_bounces, traced_paths, received_paths, row_mask]) -- tracer.py:75-79, kernel.py:38-98.
 * Traces global ray ids [ray_offset, ray_offset+n) (ray id = Warp tid; sharding keeps ids global).
 * Device outputs, each optional (NULL), rows are ray - ray_offset:
 *   traced   (n, B+1, 3) f32  kernel.py:55,88,95, NaN where the reference keeps its host NaN fill
 *   received (n, B+1, 3) f32  kernel.py:89-90, longest prefix ending at the last RX hit, NaN after
 *   row_mask (n) u32          kernel.py:91
 *   hit_kind (n, B) i32       per bounce 0 miss / 1 env / 2 receiver   (diagnostic, not in reference)
 *   hit_face (n, B) i32       per bounce face id of the chosen hit, -1 on miss (diagnostic)
 * rx may be NULL (no receiver); it is queried by brute force, so at most 65536 faces (RT_EINVAL
 * otherwise, before any launch).  max_bounces > 8 requires `traced` (it holds the path).
 * Bursts of >= 65536 rays run in a cached direction-sorted order and, from the second call with the
 * same (rays, bounces, meshes, TX) on, a cached longest-first chunk schedule; neither changes a bit
 * of the outputs (Conventions). */
int rt_trace(const rt_mesh* env, const float* tx_pos, const rt_mesh* rx, int max_bounces, int64_t ray_offset,
             int64_t n, float* traced, float* received, uint32_t* row_mask, int32_t* hit_kind, int32_t* hit_face,
             void* stream);

/* Replaces tracer.py:87 (paths[row_mask != 0]): ids of the set rows in ray order, count on device.
 * workspace: device scratch of rt_compact_workspace_bytes(n) bytes. */
int64_t rt_compact_workspace_bytes(int64_t n);
int rt_compact(const uint32_t* row_mask, int64_t n, void* workspace, int64_t workspace_bytes, int64_t* out_index,
               int64_t* out_count, void* stream);

/* Replaces tracer.py:90-117 (NaN strip, _bounce_amplitude product, float32 delay, IR accumulate).
 * received: (n, B+1, 3) device rows; index/count: output of rt_compact; max_count: host upper bound
 * of *count (grid size).  amp0 = tx_power / tx_num_rays (tracer.py:103).  impulse_response (n_bins) f64
 * is accumulated into (+=); out_bin / out_amp (max_count) optional per-path diagnostics. */
int rt_cir(const float* received, const int64_t* index, const int64_t* count, int64_t max_count, int max_bounces,
           double amp0, double light_speed, double sample_rate, int flags, int64_t n_bins, double* impulse_response,
           int32_t* out_bin, double* out_amp, void* stream);

/* The whole compute_cir hot path of one burst in two launches (tracer.py:67-117): rt_trace's
 * outputs (traced optional, received and row_mask required), then -- in one fused launch -- the
 * ordered compaction of rt_compact (out_index / *out_count, ray order) and rt_cir's impulse response,
 * which is OVERWRITTEN (zeroed, then the paths added in ray order), not accumulated.  workspace:
 * rt_trace_cir_workspace_bytes(n) bytes, 8-B aligned, zero-filled once before its first use (the
 * call leaves it ready for the next one); one workspace per stream.  n <= 2^25 rays per call. */
int64_t rt_trace_cir_workspace_bytes(int64_t n);
int rt_trace_cir(const rt_mesh* env, const float* tx_pos, const rt_mesh* rx, int max_bounces, int64_t ray_offset,
                 int64_t n, float* traced, float* received, uint32_t* row_mask, double amp0, double light_speed,
                 double sample_rate, int flags, int64_t n_bins, double* impulse_response, int64_t* out_index,
                 int64_t* out_count, void* workspace, int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- coverage (coverage.py:38-57)
 * Receiver cells on a lattice: cell (i,j,k), index (k*ny + j)*nx + i, centre
 * (x0 + i*dx, y0 + j*dy, z0 + k*dz) computed in double.  Each cell is the reference's
 * Tracer.compute_cir(tx_pos, tx_power, centre, rx_radius) followed by the signal power of
 * coverage.py:45-52; rt_coverage computes all cells exactly by shared trajectories. */
typedef struct {
  double x0, y0, z0, dx, dy, dz;
  int64_t nx, ny, nz;
} rt_grid;

typedef struct rt_coverage rt_coverage;

/* Plan a coverage run: env mesh, bounces (1..15), rays per cell (global ids ray_offset + [0,n)),
 * receiver radius; cells in x columns ix % shard_count == shard_index are computed (multi-GPU). */
int rt_coverage_create(int device, const rt_mesh* env, int max_bounces, int64_t n_rays, int64_t ray_offset,
                       const rt_grid* grid, double rx_radius, int shard_index, int shard_count, rt_coverage** out);
int rt_coverage_destroy(rt_coverage* cov);
/* Run for one transmitter.  power (n_cells f64, device): mean square of the nonzero samples of
 * np.convolve(ir, sin(2*pi*2.4e9*t), 'same') (coverage.py:45-52), NaN for a cell that receives
 * nothing, 0 for cells of other shards (sum-reduce the map across ranks).  alpha = phase step per
 * sample = (2*pi*2.4e9) * sample_window_s / (n_bins - 1).  stats[0] = candidate (cell, ray, bounce)
 * triples.  Synchronises the stream once (candidate count). */
int rt_coverage_run(rt_coverage* cov, const float* tx_pos, double tx_power, double light_speed, double sample_rate,
                    int flags, int64_t n_bins, double alpha, double* power, int64_t* stats, void* stream);
/* ---- ray-sharded coverage (multi-GPU, SURVEY §8 E1 with F2): rank r of `world` traces global ray
 * ids [ray_offset, ray_offset + n_rays) of a burst of n_rays_total rays per cell (amplitude
 * tx_power / n_rays_total, tracer.py:103) for EVERY cell, sums its first-win records per
 * (cell, bin), and sends each cell's records to the cell's owner, the rank with ix % world == rank
 * (ix = cell % nx).  The owner sums the records it receives and computes the power of its cells.
 * Replaces the per-cell loop of coverage.py:38-57 split over ranks; every rank's trajectory,
 * candidate and replay work shrinks with the rank count, and the exchange is a sparse all-to-all
 * of (cell, bin, sum) records.  Sums are exact: 192-bit unsigned fixed point, unit 2^-136, three
 * uint64 per record (least significant first), rounded once to f64 by the owner, so the map does
 * not depend on the rank count or on the order in which records arrive.
 * A record travels as one 32-B row: (cell << 32 | bin, sum word 0, 1, 2), rows 16-B aligned.
 *   1. rt_coverage_create_rays (or _create_sectors)      (once)
 *   2. rt_coverage_trace_rows_async -> rows grouped by destination rank (rank 0 first), send
 *      counts on the device; rt_coverage_trace_rows_finish -> host counts (one stream wait)
 *      (rt_coverage_records_packed fetches the rows when the caller's buffer was too small)
 *   3. all-to-all of the counts and the rows (the caller's collective: RCCL via torch.distributed)
 *   4. rt_coverage_power_packed on the received rows, segment t from rank t in source order
 *      (rt_coverage_power_rows for rows in any order, e.g. unsummed amplitudes)
 *   5. sum-reduce / all-gather of the power maps (other ranks' cells are 0 here). */
int rt_coverage_create_rays(int device, const rt_mesh* env, int max_bounces, int64_t n_rays_total, int64_t ray_offset,
                            int64_t n_rays, const rt_grid* grid, double rx_radius, int rank, int world,
                            rt_coverage** out);
/* rt_coverage_create_rays with the rays chosen by direction instead of by id: the burst of
 * n_rays_total rays sorted by the azimuth of each ray's initial direction (kernel.py:51-52) and cut
 * into 4 x world equal pieces, rank r taking pieces r, r + world, r + 2 world, r + 3 world -- four
 * wedges of directions around the transmitter, so that the rank's trajectories, candidates and
 * replays stay in few sectors of the scene while the ranks stay balanced.  Any partition of the
 * rays gives the same map bit for bit (exact fixed-point sums). */
int rt_coverage_create_sectors(int device, const rt_mesh* env, int max_bounces, int64_t n_rays_total,
                               const rt_grid* grid, double rx_radius, int rank, int world, rt_coverage** out);
/* The trace stage in two halves, so a rank can exchange its send counts on the device (the RCCL
 * all-to-all of the counts, queued on `stream`) before the host waits once for both: _async
 * queues the trajectories, candidates, exact receiver tests, replay and the exact per-(owner,
 * cell, bin) sums, writes the rows into rows_out (max_out rows) and the send counts into
 * counts_dev (device int64 [world]) without synchronising; _finish synchronises `stream` and
 * returns the host counts and stats[3] = (candidates, first-win records, 1 if rows_out held every
 * row else 0 -- then fetch them with rt_coverage_records_packed).  Returns RT_EHIP ("a look-back
 * wait timed out") if a cross-tile wait of this stage's reduce, or of the plan's previous owner
 * stage, gave up: the sums would be wrong.  Replaces the per-cell loop's trace + CIR
 * (coverage.py:43, tracer.py:63-117) for this rank's rays. */
int rt_coverage_trace_rows_async(rt_coverage* cov, const float* tx_pos, double tx_power, double light_speed,
                                 double sample_rate, int flags, int64_t n_bins, uint64_t* rows_out, int64_t max_out,
                                 int64_t* counts_dev, void* stream);
int rt_coverage_trace_rows_finish(rt_coverage* cov, int64_t* counts, int64_t* stats, void* stream);
/* The last trace stage's rows (device, 16-B aligned, max_out >= sum(counts)), when
 * rt_coverage_trace_rows_async's buffer was too small: fetched from the plan, not traced again. */
int rt_coverage_records_packed(rt_coverage* cov, uint64_t* rows_out, int64_t max_out, void* stream);
/* The owner stage (coverage.py:45-52 for this rank's cells): received rows as nseg (<= 64)
 * segments of seg_counts[t] rows (host array), segment t from rank t, merged by rank.
 * PRECONDITION: every segment strictly ascending by key -- what rt_coverage_trace_rows_async emits
 * and an all-to-all delivers.  The merge counts violations on the device (the map is then wrong);
 * rt_coverage_check reports them.  Unordered rows go through rt_coverage_power_rows (which sorts). */
int rt_coverage_power_packed(rt_coverage* cov, const uint64_t* rows, const int64_t* seg_counts, int nseg,
                             int64_t n_bins, double alpha, double* power, void* stream);
/* The owner stage on n rows in any order (keys may repeat: equal keys are summed exactly). */
int rt_coverage_power_rows(rt_coverage* cov, const uint64_t* rows, int64_t n, int64_t n_bins, double alpha,
                           double* power, void* stream);
/* Errors the device detected in this plan's earlier asynchronous stages, reported and cleared
 * (synchronises `stream`): out[0] = look-back waits that gave up (the sums of that call are wrong),
 * out[1] = received rows of a segment not in strictly ascending key order (the owner stage's
 * precondition: that power map is wrong).  RT_EHIP when either is nonzero.  out may be NULL.
 * (The owner stage returns before the device has run; Coverage.run checks after every map.) */
int rt_coverage_check(rt_coverage* cov, int64_t* out, void* stream);
/* f64 amplitudes (finite, >= 0, below 2^56) -> the exact fixed-point sums of the coverage rows
 * (truncated below 2^-136), on the device. */
int rt_coverage_amps_to_sums(const double* amps, int64_t n, uint64_t* sums, void* stream);
/* Sparse per-cell impulse responses of the last rt_coverage_run (or, ray-sharded, of this rank's cells
 * after its owner stage): keys (cell << 32 | bin) ascending, amplitudes. */
int rt_coverage_received(rt_coverage* cov, uint64_t* keys_out, double* amps_out, int64_t max_out, int64_t* n_out,
                         void* stream);
/* Signal power (same definition) of `rows` dense impulse responses (rows, n_bins) f64 on the device.
 * scratch: rows * n_bins * 16 bytes of device memory. */
int rt_power_dense(const double* impulse_responses, int64_t rows, int64_t n_bins, double alpha, void* scratch,
                   int64_t scratch_bytes, double* power, void* stream);

/* Stage timing of coverage runs (no reference counterpart: the reference prints one wall time per
 * cell, tracer.py:119).  rt_coverage_profile(cov, 1) records HIP events around the plan's kernels
 * and counts its work on every later run; rt_coverage_last_profile fills out[0..9] with the last
 * run's k_traj ms, candidate passes ms (k_cols + k_cells and the host read of their counts),
 * k_win ms, k_replay ms, reduce + power ms (sort, reduce-by-key, k_terms, k_power), whole-run ms,
 * traced ray-bounces (trajectory segments), replayed ray-bounces (sum over first-win records of
 * B - k0), candidates and first-win records.  Unrecorded entries are NaN; synchronises. */
int rt_coverage_profile(rt_coverage* cov, int enable);
/* Process-wide rt_trace / rt_trace_cir timing: rt_profile(1) (re)starts recording the start and
 * stop of every later trace kernel through its own dispatch packet (hipExtLaunchKernelGGL: no
 * marker packets in the stream) and brackets BVH ray-order sorts with events; rt_profile(k), k > 1,
 * records every k-th launch only (a launch that carries events costs the stream a few us);
 * rt_profile(0) stops.
 * rt_trace_last_profile fills out[0] = trace kernel ms, out[1] = ray-order sort ms (NaN when not
 * recorded) of the last call; rt_trace_profile_stats out = [launches, mean, min, max ms] over the
 * (last 512) kernels recorded since rt_profile(1).  Both synchronise. */
int rt_profile(int enable);
int rt_trace_profile_stats(double* out, int n);
int rt_trace_last_profile(double* out, int n);
int rt_coverage_last_profile(rt_coverage* cov, double* out, int n);

/* Self-test entry points used by the parity tests (not part of the reference surface). */
/* Debug poison: byte in 0..255 fills every coverage plan buffer and a 256 MB block of the default
 * memory pool (the stream-ordered sort workspaces come from it) with that byte before each run;
 * < 0 turns it off (default).  A result that changes with the byte reads memory the run never
 * wrote (tests/test_gpu_poison.py). */
int rt_debug_poison(int byte);
/* Debug: lists of first wins longer than n take the device-wide replay-order sort instead of the
 * 4096-entry windows (default 2^21, i.e. only one GPU's whole map; n < 0 restores it).  Process-wide.
 * The parity tests set 0 to drive the whole-map sort path on small grids. */
int rt_debug_replay_window_max(int64_t n);
int rt_selftest_math(const float* x, int64_t n, float* out, int op, void* stream);
int rt_ray_dirs(int64_t ray_offset, int64_t n, float* out, void* stream);
/* Exact fixed point of the coverage sums, on the host: op 0 converts n (w0, w1, w2) uint64 triples
 * in w to the nearest doubles in a; op 1 converts the n doubles in a to triples in w. */
int rt_selftest_fx(uint64_t* w, double* a, int64_t n, int op);
int rt_query(const rt_mesh* mesh, const float* origins, const float* dirs, int64_t n, float* t, int32_t* face,
             void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RFRT_H */
