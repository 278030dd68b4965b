// rt_bucket.h -- the exact per-(cell, bin) reduce of coverage records by fine buckets (round 5).
// Included once, by coverage.hip, after the fixed-point sums (Fx192), the segmented-sum helpers
// (SegFx) and the power parameters it uses.
//
// tracer.py:116-117 sums each bin's path amplitudes; coverage.py:38-57 does it per receiver cell.
// The device has the first-win records of a whole map (or of a rank's share of the rays) as
// (record key, amplitude) pairs in replay order, with many records per key (every ray reaching a
// cell along the same path adds to the same bin).  Until round 4 they were sorted by key with
// rocPRIM's Onesweep (3-4 passes of 10-bit digits, each a fill + a launch: ~135 us per rank of 8,
// latency-bound at that size) and summed by a look-back pass.  Here:
//
//   k_tile_reduce   per tile of 4096 records: block radix sort in LDS, equal keys summed exactly
//                   (tile-local duplicates collapse: a transmitter cell's ~125k records of one bin
//                   become one per tile), the tile's unique rows staged, and its count per fine
//                   bucket (a fixed range of cells: no cell is ever split) in a [tile][fine] matrix
//   scan            exclusive prefix of that matrix in (fine, tile) order (rocPRIM, one launch)
//   k_tile_scatter  every tile moves its staged rows to their fine bucket's region: the rows of
//                   one fine bucket are then contiguous (unsorted between tiles)
//   k_bucket        one block per range of fine buckets holding ~2048 rows: LDS radix sort of
//                   the range by key, exact sums of the remaining duplicates (across tiles), the
//                   unique position by a ticketed decoupled look-back, then per mode: the send rows
//                   and owner bounds of a ray-sharded rank, or the power terms and cell ranges
//
// The owner stage of a ray-sharded map receives sorted segments (one per source rank): there
// k_seg_bounds finds every fine bucket's range in every segment (lockstep binary searches), and
// k_bucket gathers a block's rows from the segments directly -- no tile pass, no merge kernel.
//
// Every sum is the integer Fx192 sum, so neither the tiling, the bucketing, nor the order in which
// tiles land in a region can change a bit: the outputs equal the sort-based reduce's exactly
// (tests/test_gpu_coverage.py, tests/test_gpu_fullsize.py).  A range holding more rows than the
// block's LDS capacity is processed in key-ordered rounds (bisection on the key; slow but exact,
// and never reached by the benched maps: the tile pass already collapsed the hot keys).
#pragma once

constexpr int kBkThreads = 1024, kBkItems = 4, kBkTile = kBkThreads * kBkItems;  // 4096 rows per tile / block
constexpr int kBkMaxFine = 8192;   // fine buckets (LDS histogram of k_tile_reduce: 32 KB)
constexpr int kBkTarget = 2048;    // rows per k_bucket block (the T-split of the fine buckets' prefix)
constexpr int kBkMaxSegs = 64;

// ---- keys.  Compact record keys (record_key) are [owner | cell | bin] (owner-local cell when
// ray-sharded); received rows carry wide keys (cell << 32 | bin) with global cells.  A fine bucket
// is `1 << cs` consecutive (owner-local) cells, all bins; its id is the key's local value >> fshift.
struct BkKeys {
  int bin_bits, cs;      // fine bucket = (local cell) >> cs
  int cell_bits;         // compact keys: the owner field starts at bin_bits + cell_bits
  int wide_in;           // 1: rows carry wide keys with global cells (owner stage); 0: compact keys
  int64_t nx;            // wide_in: cell -> owner-local cell (row * nxo + ix / world)
  int world, owner;
  WideKey wk;            // compact key -> output wide key (owner << own_shift | cell << 32 | bin)
  // the sort key; ~0 stays ~0.  32-bit index arithmetic (cells < 2^32, rt_coverage_create): a 64-bit
  // division by a run-time divisor is a ~100-instruction sequence on every row
  __device__ __forceinline__ uint64_t local(uint64_t k) const {
    if (!wide_in || k == ~0ull) return k;
    const uint32_t cell = (uint32_t)(k >> 32);
    const uint64_t bin = k & 0xFFFFFFFFull;
    uint32_t lc = cell;
    if (world > 1) {
      const uint32_t n = (uint32_t)nx, w = (uint32_t)world, row = cell / n, ix = cell - row * n;
      lc = row * ((n + w - 1) / w) + ix / w;
    }
    return (uint64_t)lc << bin_bits | bin;
  }
  __device__ __forceinline__ bool foreign(uint64_t k) const {  // wide key of another owner's cell
    if (!wide_in || world <= 1) return false;
    const uint32_t cell = (uint32_t)(k >> 32), n = (uint32_t)nx;
    return (cell % n) % (uint32_t)world != (uint32_t)owner;
  }
  __device__ __forceinline__ uint64_t wide(uint64_t k) const { return wide_in ? k : wk(k); }
  __device__ __forceinline__ int fine(uint64_t lk) const { return (int)(lk >> (bin_bits + cs)); }
};

// ---- block-wide exact sums of runs of equal keys, over items sorted ascending across the block in
// blocked arrangement (thread t holds items t*I .. t*I+I-1); invalid items carry ~0 and come last.
// end[j]: item j is the last of its run (and valid); sum[j]: the run's exact sum there; uidx[j]: the
// run's index among the block's runs.  Returns the block's run count.
template <int I>
struct BkRunScratch {
  uint64_t first[kBkThreads], last[kBkThreads];
  SegFx wseg[kBkThreads / 64];
  int wcnt[kBkThreads / 64];
};
template <int I>
__device__ __forceinline__ int block_runs(const uint64_t (&k)[I], const Fx192 (&v)[I], bool (&end)[I],
                                          Fx192 (&sum)[I], int (&uidx)[I], BkRunScratch<I>& sc) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const Fx192 zero{0, 0, 0};
  sc.first[tid] = k[0];
  sc.last[tid] = k[I - 1];
  __syncthreads();
  const uint64_t prev0 = tid > 0 ? sc.last[tid - 1] : ~0ull;
  const uint64_t next_last = tid + 1 < kBkThreads ? sc.first[tid + 1] : ~0ull;
  bool head[I];
  SegFx th{false, zero};
  int c = 0;
#pragma unroll
  for (int j = 0; j < I; ++j) {
    const bool valid = k[j] != ~0ull;
    const uint64_t p = j ? k[j - 1] : prev0;
    const uint64_t nx = j + 1 < I ? k[j + 1] : next_last;
    head[j] = valid && (tid == 0 && j == 0 ? true : p != k[j]);
    end[j] = valid && nx != k[j];
    c += end[j] ? 1 : 0;
    th = seg_op(th, SegFx{head[j], valid ? v[j] : zero});
  }
  // inclusive wave scans: segmented sums and run-end counts
  SegFx sx = th;
  int x = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const SegFx sy = shfl_up_seg(sx, o);
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) {
      sx = seg_op(sy, sx);
      x += y;
    }
  }
  if (lane == 63) {
    sc.wseg[w] = sx;
    sc.wcnt[w] = x;
  }
  SegFx lx = shfl_up_seg(sx, 1);
  if (lane == 0) lx = SegFx{false, zero};
  __syncthreads();
  SegFx pre{false, zero};
  int before = x - c, total = 0;
  for (int q = 0; q < kBkThreads / 64; ++q) {
    if (q < w) {
      pre = seg_op(pre, sc.wseg[q]);
      before += sc.wcnt[q];
    }
    total += sc.wcnt[q];
  }
  pre = seg_op(pre, lx);
  Fx192 acc = pre.t;  // the sum of the run open before this thread's first item
  int u = before;
#pragma unroll
  for (int j = 0; j < I; ++j) {
    acc = head[j] ? v[j] : FxPlus()(acc, v[j]);
    sum[j] = acc;
    uidx[j] = u;
    u += end[j] ? 1 : 0;
  }
  __syncthreads();  // the scratch is reused by the caller's next call
  return total;
}

// ---------------------------------------------------------------- 1. tiles
struct TileArgs {
  const uint64_t* keys;  // compact record keys (~0: dropped), replay order
  const double* amps;
  int64_t n;
  int fshift, fbits;     // fine bucket = key >> fshift, nf = 2^fbits buckets
  int64_t ntiles;
  uint64_t* stage;       // [ntiles * 4096][4]: the tile's unique (key, sum) rows, grouped by fine bucket
  int32_t* tcnt;         // [ntiles][nf]: the tile's unique rows per fine bucket
  int32_t* tuniq;        // [ntiles]
  unsigned long long* ticket;  // zeroed for k_bucket (stream order: it runs later)
};
// The tile is sorted on 16 bits only -- its rows' fine bucket, then a hash of the full key -- in two
// 8-bit radix passes instead of five on the 35-bit key: rows end up grouped by fine bucket (what
// k_tile_scatter needs), and equal keys adjacent unless another key of the same bucket and hash
// falls between them, which leaves a duplicate for k_bucket to add (sums are exact either way).
__global__ __launch_bounds__(kBkThreads) void k_tile_reduce(TileArgs a) {
  using Sort = rocprim::block_radix_sort<uint32_t, kBkThreads, kBkItems, uint16_t>;
  __shared__ union {
    typename Sort::storage_type sort;
    BkRunScratch<kBkItems> runs;
  } sm;
  __shared__ int32_t s_cnt[kBkMaxFine];
  const int tid = threadIdx.x;
  const int64_t tile = blockIdx.x, t0 = tile * kBkTile;
  if (tile == 0 && tid == 0 && a.ticket) *a.ticket = 0ull;
  const int nf = 1 << a.fbits, hb = 15 - a.fbits;
  for (int f = tid; f < nf; f += kBkThreads) s_cnt[f] = 0;
  uint32_t sk[kBkItems];
  uint16_t ix[kBkItems];
#pragma unroll
  for (int j = 0; j < kBkItems; ++j) {
    const int q = tid * kBkItems + j;
    const int64_t i = t0 + q;
    const uint64_t key = i < a.n ? a.keys[i] : ~0ull;
    const uint32_t h = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - hb));
    sk[j] = key == ~0ull ? (1u << 15) : ((uint32_t)(key >> a.fshift) << hb | h);
    ix[j] = (uint16_t)q;
  }
  Sort().sort(sk, ix, sm.sort, 0, 16);
  __syncthreads();
  uint64_t k[kBkItems];
  Fx192 v[kBkItems], sum[kBkItems];
  bool end[kBkItems];
  int uidx[kBkItems];
#pragma unroll
  for (int j = 0; j < kBkItems; ++j) {
    const int64_t i = t0 + ix[j];
    const bool ok = sk[j] != (1u << 15);
    k[j] = ok ? a.keys[i] : ~0ull;
    v[j] = ok ? fx_from_double(a.amps[i]) : Fx192{0, 0, 0};
  }
  const int total = block_runs<kBkItems>(k, v, end, sum, uidx, sm.runs);
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int j = 0; j < kBkItems; ++j) {
    if (!end[j]) continue;
    u64x2* row = reinterpret_cast<u64x2*>(a.stage + 4 * (t0 + uidx[j]));
    row[0] = u64x2{k[j], sum[j].w0};
    row[1] = u64x2{sum[j].w1, sum[j].w2};
    atomicAdd(&s_cnt[(int)(k[j] >> a.fshift)], 1);
  }
  __syncthreads();
  for (int f = tid; f < nf; f += kBkThreads) a.tcnt[tile * nf + f] = s_cnt[f];
  if (tid == 0) a.tuniq[tile] = total;
}

// the [tile][fine] counts read in (fine, tile) order, and a trailing 0 (the scan's last output is
// the total): the input of rocprim::exclusive_scan
struct TileCountsFT {
  const int32_t* tcnt;
  int64_t ntiles;
  int nf;
  __host__ __device__ int32_t operator()(uint32_t q) const {
    const int64_t f = (int64_t)q / ntiles, t = (int64_t)q - f * ntiles;
    return f < nf ? tcnt[t * nf + f] : 0;
  }
};

// ---------------------------------------------------------------- 2. fine-bucket regions
struct ScatterArgs {
  const uint64_t* stage;
  const int32_t* tuniq;
  const int32_t* pos;  // [nf][ntiles] exclusive prefix (+ the total at [nf * ntiles])
  int64_t ntiles;
  int fshift, nf;
  uint64_t* rows;      // [total][4]
  int64_t* fs;         // [nf + 1] region starts (written by tile 0)
  int32_t* blk_f0;     // [nblocks + 1]: k_bucket block p's first bucket (written by tile 0)
  int nblocks;
};
__global__ __launch_bounds__(kBkThreads) void k_tile_scatter(ScatterArgs a) {
  __shared__ int32_t s_first[kBkMaxFine];
  __shared__ uint16_t s_f[kBkTile];
  const int tid = threadIdx.x;
  const int64_t tile = blockIdx.x;
  if (tile == 0) {
    // region starts, and k_bucket block p's first bucket: the first f with fs[f] >= p T, i.e. the
    // blocks p with fs[f - 1] < p T <= fs[f] start at f (blocks past the total start at nf)
    const int64_t total = a.pos[(int64_t)a.nf * a.ntiles];
    for (int f = tid; f <= a.nf; f += kBkThreads) {
      const int64_t fsf = a.pos[(int64_t)f * a.ntiles];
      a.fs[f] = fsf;
      const int64_t plo = f == 0 ? 0 : a.pos[(int64_t)(f - 1) * a.ntiles] / kBkTarget + 1;
      const int64_t phi = f == a.nf ? a.nblocks : fsf / kBkTarget;
      for (int64_t p = plo; p <= phi && p <= a.nblocks; ++p) a.blk_f0[p] = f;
    }
    (void)total;
  }
  const int nu = a.tuniq[tile];
  const uint64_t* st = a.stage + 4 * tile * kBkTile;
  for (int u = tid; u < nu; u += kBkThreads) s_f[u] = (uint16_t)(st[4 * u] >> a.fshift);
  __syncthreads();
  for (int u = tid; u < nu; u += kBkThreads)
    if (u == 0 || s_f[u - 1] != s_f[u]) s_first[s_f[u]] = u;
  __syncthreads();
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  for (int u = tid; u < nu; u += kBkThreads) {
    const int f = s_f[u];
    const int64_t dst = a.pos[(int64_t)f * a.ntiles + tile] + (u - s_first[f]);
    const u64x2* src = reinterpret_cast<const u64x2*>(st + 4 * u);
    u64x2* d = reinterpret_cast<u64x2*>(a.rows + 4 * dst);
    d[0] = src[0];
    d[1] = src[1];
  }
}

// Owner stage: every fine bucket's first row in every received segment (each segment sorted by
// wide key): lb[s][f] = first row of segment s whose owner-local fine id is >= f, f = 0..nf; the
// nseg searches of a bucket boundary run in lockstep (independent loads per step).  fs[f] = the
// rows of all segments before bucket f.
struct SegBoundsArgs {
  unsigned long long* ticket;  // zeroed for k_bucket (stream order)
  const uint64_t* rows;  // received (key, sum) rows, stride 4 (key first)
  int64_t off[kBkMaxSegs + 1];
  int nseg, steps;
  BkKeys kk;
  int nf;
  int64_t* lb;   // [nseg][nf + 1]
  int64_t* fs;   // [nf + 1]
};
template <int NS>
__global__ __launch_bounds__(256) void k_seg_bounds(SegBoundsArgs a) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f == 0 && a.ticket) *a.ticket = 0ull;
  if (f > a.nf) return;
  const uint64_t bound = (uint64_t)f << (a.kk.bin_bits + a.kk.cs);  // first local key of bucket f
  int64_t lo[NS], len[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    lo[s] = s < a.nseg ? a.off[s] : 0;
    len[s] = s < a.nseg ? a.off[s + 1] - a.off[s] : 0;
  }
  for (int st = 0; st < a.steps; ++st) {
    uint64_t km[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) km[s] = len[s] > 0 ? a.rows[4 * (lo[s] + (len[s] >> 1))] : 0ull;  // independent loads
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (len[s] <= 0) continue;
      const int64_t half = len[s] >> 1;
      const bool right = a.kk.local(km[s]) < bound;
      lo[s] = right ? lo[s] + half + 1 : lo[s];
      len[s] = right ? len[s] - half - 1 : half;
    }
  }
  int64_t tot = 0;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (s >= a.nseg) continue;
    a.lb[(int64_t)s * (a.nf + 1) + f] = lo[s];
    tot += lo[s] - a.off[s];
  }
  a.fs[f] = tot;
}

// ---------------------------------------------------------------- 3. buckets
enum BkMode { kBkSend = 0, kBkPower = 1 };
struct BucketArgs {
  // rows: (key, sum words 0..2), stride 4.  nseg == 0: one region, rows[fs[f0] .. fs[f1]); else
  // segment s of the owner stage holds rows[lb[s][f0] .. lb[s][f1])
  const uint64_t* rows;
  const int64_t* fs;
  const int64_t* lb;
  const int32_t* blk_f0;  // nseg == 0: block p's buckets [blk_f0[p], blk_f0[p + 1]) (k_tile_scatter)
  int nseg;
  int nf;
  BkKeys kk;
  int cap;               // rows per round (<= kBkTile; smaller only to exercise the rounds in tests)
  // look-back over blocks in ticket order (tickets zeroed earlier in stream order; states tagged)
  uint64_t* states;
  unsigned long long* ticket;
  uint64_t tag;
  unsigned* errors;
  int64_t* nuniq;
  // both modes: the reduced records (wide keys, exact sums, f64)
  uint64_t* ukeys;
  Fx192* usums;
  double* uamps;
  // kBkSend: the rows for the owners (owner stripped from the key) -- packed 32-B rows in `out`, or
  // keys in `out` and sums in `sums_out` -- while they fit out_cap; bounds[o] = first row of owner o
  uint64_t* out;
  Fx192* sums_out;
  int packed;
  int64_t out_cap;
  int64_t* bounds;
  int world, own_shift;
  // kBkPower: terms and cell ranges (the inputs of k_power_small / k_power)
  double *tcos, *tsin, *ev;
  int64_t ncell;
  int32_t *cstart, *cend, *cepoch;
  int32_t epoch;
  unsigned* nbig;
  PowerParams P;
};
struct BkScratch {
  int64_t segoff[kBkMaxSegs + 1];  // prefix of the block's rows per segment
  int64_t seglo[kBkMaxSegs];       // first row of the block's part of each segment
  int f0, f1;
  int64_t prefix;                  // the block's first unique index (look-back)
  int32_t carry;                   // the last cell of the previous round (kBkPower)
  int red[kBkThreads / 64];
  int64_t red64[kBkThreads / 64];
  uint32_t tile;
};

// row index of the block's item q (0 <= q < its row count)
__device__ __forceinline__ int64_t bk_row(const BucketArgs& a, const BkScratch& s, int64_t q) {
  if (a.nseg == 0) return s.seglo[0] + q;
  int lo = 0, hi = a.nseg - 1;  // the last segment with segoff <= q
  while (lo < hi) {
    const int m = (lo + hi + 1) >> 1;
    if (s.segoff[m] <= q) lo = m;
    else hi = m - 1;
  }
  return s.seglo[lo] + (q - s.segoff[lo]);
}
__device__ __forceinline__ int64_t bk_sum(int64_t v, BkScratch& s) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s.red64[threadIdx.x >> 6] = v;
  __syncthreads();
  int64_t t = 0;
  for (int q = 0; q < kBkThreads / 64; ++q) t += s.red64[q];
  __syncthreads();
  return t;
}

// One block per range of fine buckets (T-split: block p takes the buckets whose rows start in
// [p T, (p + 1) T) of the regions' prefix; every bucket belongs to exactly one block and a cell to
// exactly one bucket).  Rows of a range are sorted by local key in LDS and equal keys summed; the
// block's first unique index comes from the look-back; then per mode the uniques are written.
#ifndef RT_BK_RADIX
#define RT_BK_RADIX 8
#endif
template <int MODE>
__global__ __launch_bounds__(kBkThreads) void k_bucket(BucketArgs a) {
  using Sort = rocprim::block_radix_sort<uint64_t, kBkThreads, kBkItems, uint32_t, 1, 1, RT_BK_RADIX>;
  __shared__ union {
    typename Sort::storage_type sort;
    BkRunScratch<kBkItems> runs;
    struct {
      uint64_t lk[kBkTile];
      uint32_t q[kBkTile];
    } sel;  // a round's selected items (ranges above the capacity)
  } sm;
  __shared__ BkScratch s;
  __shared__ int32_t s_ucell[kBkTile];  // per unique of a round: its cell (power) or fine bucket (send)
  __shared__ uint64_t s_lk[kBkTile];    // owner stage: the block's local keys in row order (merge)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) s.tile = (uint32_t)atomicAdd(a.ticket, 1ull);
  __syncthreads();
  const int64_t p = s.tile;
  if (tid < 2) {  // first bucket f in [0, nf] with fs[f] >= (p + tid) T (fs[nf] = the total)
    int lo = 0;
    if (a.blk_f0) {
      lo = a.blk_f0[p + tid];
    } else {
      const int64_t target = (p + tid) * kBkTarget;
      int hi = a.nf;
      while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (a.fs[m] < target) lo = m + 1;
        else hi = m;
      }
    }
    if (tid == 0) s.f0 = lo;
    else s.f1 = lo;
  }
  __syncthreads();
  const int f0 = s.f0, f1 = s.f1;
  if (tid == 0) {
    if (a.nseg == 0) {
      s.seglo[0] = a.fs[f0];
      s.segoff[0] = 0;
      s.segoff[1] = a.fs[f1] - a.fs[f0];
    } else {
      int64_t acc = 0;
      for (int g = 0; g < a.nseg; ++g) {
        const int64_t b0 = a.lb[(int64_t)g * (a.nf + 1) + f0], b1 = a.lb[(int64_t)g * (a.nf + 1) + f1];
        s.seglo[g] = b0;
        s.segoff[g] = acc;
        if (b1 >= b0) acc += b1 - b0;
        else atomicAdd(a.errors + 1, 1u);  // a segment not in key order (its bounds are not monotone)
      }
      s.segoff[a.nseg] = acc;
    }
    s.carry = -1;
  }
  __syncthreads();
  const int64_t count = s.segoff[a.nseg == 0 ? 1 : a.nseg];
  const int fsh = a.kk.bin_bits + a.kk.cs;
  const uint64_t base = (uint64_t)f0 << fsh;
  const uint64_t span = (uint64_t)(f1 - f0) << fsh;  // local keys - base lie in [0, span)
  int eb = 1;
  while (eb < 62 && (1ull << eb) < span) ++eb;
  const uint64_t kend = 1ull << eb;
  const Fx192 zero{0, 0, 0};
  // kBkSend: owner o's first bucket is o << obits (the owner field sits above the cell field)
  const int obits = a.kk.cell_bits - a.kk.cs;

  // One round: the block's rows with local key in [lo, hi) (all of them when `all`), sorted, equal
  // keys summed; when `emit`, the uniques are written from index out_base.  Returns their count.
  auto round = [&](uint64_t lo, uint64_t hi, bool all, bool emit, int64_t out_base) -> int {
    uint64_t k[kBkItems];
    uint32_t q[kBkItems];
    bool sorted = false;
    if (all && a.nseg > 0) {
      // owner stage: the block's rows are nseg sorted pieces (one per source segment); their merge
      // by (key, segment) is each row's index in its piece plus, in every other piece, the rows
      // with a smaller key (or an equal one, for the pieces before it) -- binary searches in LDS
      // instead of a radix sort
      bool bad = false;
      for (int64_t qq = tid; qq < count; qq += kBkThreads) {
        const uint64_t rk = a.rows[4 * bk_row(a, s, qq)];
        const uint64_t lk = a.kk.local(rk) - base;
        s_lk[qq] = lk;
        bad = bad || lk >= span || a.kk.foreign(rk);
      }
      if (emit && bad) atomicAdd(a.errors + 1, 1u);
      __syncthreads();
      for (int64_t qq = tid; qq < count; qq += kBkThreads) {
        int g = 0;
        while (g + 1 < a.nseg && s.segoff[g + 1] <= qq) ++g;
        const uint64_t key = s_lk[qq];
        int64_t rank = qq - s.segoff[g];
        for (int h = 0; h < a.nseg; ++h) {
          if (h == g) continue;
          int64_t l = s.segoff[h], r = s.segoff[h + 1];
          while (l < r) {
            const int64_t m = (l + r) >> 1;
            const uint64_t km = s_lk[m];
            if (km < key || (h < g && km == key)) l = m + 1;
            else r = m;
          }
          rank += l - s.segoff[h];
        }
        sm.sel.lk[rank] = key;
        sm.sel.q[rank] = (uint32_t)qq;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < kBkItems; ++j) {
        const int r = tid * kBkItems + j;
        k[j] = r < count ? sm.sel.lk[r] : ~0ull;
        q[j] = r < count ? sm.sel.q[r] : 0u;
      }
      __syncthreads();
      sorted = true;
    } else if (all) {
      bool bad = false;
#pragma unroll
      for (int j = 0; j < kBkItems; ++j) {
        const int64_t qq = (int64_t)tid * kBkItems + j;
        k[j] = ~0ull;
        if (qq < count) {
          const uint64_t rk = a.rows[4 * bk_row(a, s, qq)];
          k[j] = a.kk.local(rk) - base;
          // received rows (owner stage): a row of another owner's cell, or outside the block's
          // buckets (a segment not in ascending key order), would be summed into a wrong cell
          if (a.kk.wide_in && (k[j] >= span || a.kk.foreign(rk))) bad = true;
        }
        q[j] = (uint32_t)qq;
      }
      if (emit && bad) atomicAdd(a.errors + 1, 1u);
    } else {  // the selected rows, compacted into LDS in row order
      int nsel = 0;
      for (int64_t c0 = 0; c0 < count; c0 += kBkThreads) {
        const int64_t qq = c0 + tid;
        uint64_t lk = 0;
        bool in = false;
        if (qq < count) {
          lk = a.kk.local(a.rows[4 * bk_row(a, s, qq)]) - base;
          in = lk >= lo && lk < hi;
        }
        const uint64_t m = __ballot(in);
        if (lane == 0) s.red[w] = __popcll(m);
        __syncthreads();
        int off = nsel, tot = 0;
        for (int g = 0; g < kBkThreads / 64; ++g) {
          off += g < w ? s.red[g] : 0;
          tot += s.red[g];
        }
        if (in) {
          const int r = off + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          sm.sel.lk[r] = lk;
          sm.sel.q[r] = (uint32_t)qq;
        }
        nsel += tot;
        __syncthreads();
      }
#pragma unroll
      for (int j = 0; j < kBkItems; ++j) {
        const int r = tid * kBkItems + j;
        k[j] = r < nsel ? sm.sel.lk[r] : ~0ull;
        q[j] = r < nsel ? sm.sel.q[r] : 0u;
      }
      __syncthreads();
    }
    if (!sorted) Sort().sort(k, q, sm.sort, 0, (unsigned)eb);
    __syncthreads();
    Fx192 v[kBkItems], sum[kBkItems];
    bool end[kBkItems];
    int uidx[kBkItems];
#pragma unroll
    for (int j = 0; j < kBkItems; ++j) {
      v[j] = zero;
      if (k[j] != ~0ull) {
        const uint64_t* r = a.rows + 4 * bk_row(a, s, (int64_t)q[j]);
        v[j] = Fx192{r[1], r[2], r[3]};
      }
    }
    const int nu = block_runs<kBkItems>(k, v, end, sum, uidx, sm.runs);
    if (!emit) return nu;
    typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
    const uint64_t omask = MODE == kBkSend ? (1ull << a.own_shift) - 1 : ~0ull;
#pragma unroll
    for (int j = 0; j < kBkItems; ++j) {
      if (!end[j]) continue;
      const int64_t u = out_base + uidx[j];
      const uint64_t lk = k[j] + base;
      uint64_t wkey;
      if (a.kk.wide_in) {  // owner-local cell -> the global cell of the wide key
        const uint64_t lc = lk >> a.kk.bin_bits, bin = lk & ((1ull << a.kk.bin_bits) - 1);
        uint64_t cell = lc;
        if (a.kk.world > 1) {
          const uint32_t w = (uint32_t)a.kk.world, n = (uint32_t)a.kk.nx, nxo = (n + w - 1) / w;
          const uint32_t l32 = (uint32_t)lc, row = l32 / nxo;
          cell = (uint64_t)row * n + (uint64_t)(l32 - row * nxo) * w + (uint32_t)a.kk.owner;
        }
        wkey = cell << 32 | bin;
      } else {
        wkey = a.kk.wk(lk);
      }
      const double amp = fx_to_double(sum[j]);
      a.ukeys[u] = wkey;
      if (a.usums) a.usums[u] = sum[j];
      a.uamps[u] = amp;
      if constexpr (MODE == kBkSend) {
        if (a.out && u < a.out_cap) {
          if (a.packed) {
            u64x2* row = reinterpret_cast<u64x2*>(a.out + 4 * u);
            row[0] = u64x2{wkey & omask, sum[j].w0};
            row[1] = u64x2{sum[j].w1, sum[j].w2};
          } else {
            a.out[u] = wkey & omask;
            a.sums_out[u] = sum[j];
          }
        }
        s_ucell[uidx[j]] = a.kk.fine(lk);
      } else {
        const PowerParams& P = a.P;
        const int64_t m = (int64_t)(wkey & 0xFFFFFFFFull);
        double sp, cp;
        sincos_turns(P.turns * (double)(P.half - m), sp, cp);
        a.tcos[u] = amp * cp;
        a.tsin[u] = amp * sp;
        const int64_t st = m - P.half > 0 ? m - P.half : 0;
        const int64_t en = m + (P.n_bins - 1 - P.half), e1 = (en < P.n_bins - 1 ? en : P.n_bins - 1) + 1;
        sincos_turns(P.turns * (double)st, a.ev[4 * u], a.ev[4 * u + 1]);
        sincos_turns(P.turns * (double)e1, a.ev[4 * u + 2], a.ev[4 * u + 3]);
        s_ucell[uidx[j]] = (int32_t)(wkey >> 32);
      }
    }
    __syncthreads();
    if constexpr (MODE == kBkSend) {
      // bounds[o] for the owners whose first bucket lies in this block's range and whose first
      // local key falls in this round: the first unique at or after that bucket
      for (int o = tid; o < a.world; o += kBkThreads) {
        const int fo = o << obits;
        if (fo < f0 || fo >= f1) continue;
        const uint64_t lko = (uint64_t)(fo - f0) << fsh;
        if (lko < lo || lko >= hi) continue;
        int l = 0, r = nu;  // first unique with fine id >= fo
        while (l < r) {
          const int mm = (l + r) >> 1;
          if (s_ucell[mm] < fo) l = mm + 1;
          else r = mm;
        }
        a.bounds[o] = out_base + l;
      }
    } else {
      // cell ranges (cells never straddle fine buckets, so never blocks; a cell may span rounds:
      // its first round writes cstart, each later one rewrites cend)
      const int32_t carry = s.carry;
      for (int uu = tid; uu < nu; uu += kBkThreads) {
        const int32_t cur = s_ucell[uu];
        if (cur < 0 || cur >= a.ncell) continue;
        const int64_t u = out_base + uu;
        if (uu == 0 ? carry != cur : s_ucell[uu - 1] != cur) {
          a.cstart[cur] = (int32_t)u;
          a.cepoch[cur] = a.epoch;
        }
        if (uu + 1 == nu || s_ucell[uu + 1] != cur) a.cend[cur] = (int32_t)(u + 1);
      }
    }
    __syncthreads();
    if (tid == 0 && nu > 0) s.carry = s_ucell[nu - 1];
    __syncthreads();
    return nu;
  };

  // ranges above the capacity: key-ordered rounds [lo, hi) of <= cap rows (bisection on the key)
  const int64_t cap = a.cap;
  auto count_in = [&](uint64_t lo, uint64_t hi) -> int64_t {
    int64_t c = 0;
    for (int64_t qq = tid; qq < count; qq += kBkThreads) {
      const uint64_t lk = a.kk.local(a.rows[4 * bk_row(a, s, qq)]) - base;
      c += (lk >= lo && lk < hi) ? 1 : 0;
    }
    return bk_sum(c, s);
  };
  auto next_hi = [&](uint64_t lo) -> uint64_t {  // the largest hi with <= cap rows in [lo, hi)
    if (count_in(lo, kend) <= cap) return kend;
    uint64_t hi = lo;
    for (int b = eb - 1; b >= 0; --b) {
      const uint64_t cand = hi + (1ull << b);
      if (cand <= kend && count_in(lo, cand) <= cap) hi = cand;
    }
    return hi;
  };
  const bool one = count <= cap;
  int64_t nb = 0;  // the block's uniques
  if (f0 < f1) {
    if (one) {
      nb = round(0, kend, true, false, 0);
    } else {
      if (a.kk.wide_in) {  // received rows: the checks of round()'s one-pass path, once for all rounds
        int64_t bad = 0;
        for (int64_t qq = tid; qq < count; qq += kBkThreads) {
          const uint64_t rk = a.rows[4 * bk_row(a, s, qq)];
          const uint64_t lk = a.kk.local(rk) - base;
          bad += (lk >= span || a.kk.foreign(rk)) ? 1 : 0;
        }
        if (bk_sum(bad, s) && tid == 0) atomicAdd(a.errors + 1, 1u);
      }
      for (uint64_t lo = 0; lo < kend;) {
        const uint64_t hi = next_hi(lo);
        if (hi <= lo) {  // one key with more than cap rows: impossible (<= 1 per tile, tiles <= cap)
          if (tid == 0) atomicAdd(a.errors, 1u);
          break;
        }
        nb += round(lo, hi, false, false, 0);
        lo = hi;
      }
    }
  }
  // look-back over the blocks in ticket order (= bucket order): the block's first unique index
  if (w == 0) {
    uint64_t* st = a.states + p;
    if (lane == 0)
      __hip_atomic_store(st, a.tag | (p == 0 ? kOwnInc : kOwnAgg) | (uint64_t)nb, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    uint64_t excl = 0;
    if (p > 0) {
      int spins = 0;
      for (int64_t jbase = p - 1;;) {
        const int64_t j = jbase - lane;
        const uint64_t sv = j >= 0 ? __hip_atomic_load(a.states + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        const bool ready = j < 0 || (sv & kOwnTagMask) == a.tag;
        const uint64_t incm = __ballot(j >= 0 && ready && (sv & kOwnInc) != 0);
        const int stop = incm ? __builtin_ctzll(incm) : 63;
        const uint64_t used = stop == 63 ? ~0ull : ((2ull << stop) - 1);
        if (__ballot(!ready) & used) {
          if (++spins > (1 << 22)) {
            if (lane == 0) atomicAdd(a.errors, 1u);
            break;
          }
          continue;
        }
        uint64_t cnt = (j >= 0 && lane <= stop) ? (sv & kOwnCount) : 0ull;
        for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
        excl += cnt;
        if (incm || jbase < 64) break;  // block 0 always publishes an inclusive state
        jbase -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(st, a.tag | kOwnInc | (excl + (uint64_t)nb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s.prefix = (int64_t)excl;
      if (f1 == a.nf && f0 < f1) {  // the block holding the last bucket: the totals
        *a.nuniq = (int64_t)excl + nb;
        if (MODE == kBkSend) a.bounds[a.world] = (int64_t)excl + nb;
      }
      if (MODE == kBkPower && p == 0) *a.nbig = 0u;  // k_power_small lists the big cells afresh
    }
  }
  __syncthreads();
  if (f0 >= f1) return;
  if (one) {
    round(0, kend, true, true, s.prefix);
  } else {
    int64_t o = s.prefix;
    for (uint64_t lo = 0; lo < kend;) {
      const uint64_t hi = next_hi(lo);
      if (hi <= lo) break;
      o += round(lo, hi, false, true, o);
      lo = hi;
    }
  }
}
