// Host-side launcher API of the wormhole_amd HIP kernels.
//
// Every launcher takes raw device pointers plus the HIP stream to enqueue on;
// none allocates, frees or synchronises, so every call is hipGraph-capturable.
// The torch binding layer (csrc/bind/hip_ops.cc) validates shapes/dtypes and
// passes the current PyTorch HIP stream.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wh {

// ---------------------------------------------------------------- scan.hip
// exclusive prefix sum: out[i] = sum_{k<i} in[k], out[n] = total.
// tmp must hold scan_tmp_elems(n) int64.
int64_t scan_tmp_elems(int64_t n);
void scan_i32(const int32_t* in, int64_t* out, int64_t n, int64_t* tmp, hipStream_t s);
void scan_i64(const int64_t* in, int64_t* out, int64_t n, int64_t* tmp, hipStream_t s);
// Decoupled look-back state (device side in wh_lookback.h).
constexpr int kLbMaxTiles = 1 << 16;
constexpr int kLbChannels = 2;
struct Lookback {
  unsigned long long* gran;  // [kLbChannels][kLbMaxTiles] {tag, value} granules
  unsigned int* ticket;      // [1], zero between launches
  unsigned int* err;         // [1], sticky spin-timeout flag
  unsigned int epoch;        // 1 .. 2^30-1, new per launch
};
// Workspace of the single-pass look-back scans (wh_lookback.h): ONE per
// device, zero-initialised once, shared by every fused-scan kernel on the
// device's compute stream. lookback_bind hands out a fresh epoch per launch.
int64_t lookback_ws_words();  // uint64 words
Lookback lookback_bind(void* ws);

// ------------------------------------------------------------ localize.hip
// Batch-local de-duplication of uint64 feature ids (reference Localizer,
// learn/base/localizer.h:42-221) via a device open-addressing table of
// `tsize` (power of two) slots, then a radix sort of (local id, position)
// pairs on ceil(log2 U) bits for the CSC. The host sizes the table from the
// previous minibatch's unique count; if it fills up, inserts give up after a
// full probe cycle and count into overflow[0] so the host retries with
// tsize >= 2*nnz (which cannot overflow). tkeys[tsize] (init ~0) is scratch.
void loc_insert(const uint64_t* keys, int64_t nnz, uint64_t* tkeys, int64_t tsize,
                int32_t* slot_of, int64_t* overflow, hipStream_t s);
// keys[i] %= m (uint64): the ps-lite max_key key-space folding applied by
// the reference Localizer (learn/base/localizer.h:108-115)
void key_mod(uint64_t* keys, int64_t n, uint64_t m, hipStream_t s);
// per-owner counts of the occupied slots (owner = mix64b(key) % nshard):
// blkcnt [nshard * loc_owner_blocks(tsize)] becomes the owner-major exclusive
// scan of the per-block counts (= blkoff for loc_assign); owner_cnt[0..nshard)
// and owner_cnt[nshard] = *overflow, which is reset to 0.
int64_t loc_owner_blocks(int64_t tsize);
void loc_owner_count(const uint64_t* tkeys, int64_t tsize, int nshard, int64_t* blkcnt,
                     int64_t* owner_cnt, int64_t* overflow, hipStream_t s);
// assign local ids grouped by owner. Writes tlid[slot], uniq[lid] and
// empties every slot it read, so a persistent table needs no clearing pass.
void loc_assign(uint64_t* tkeys, int64_t tsize, int nshard, const int64_t* blkoff,
                int32_t* tlid, uint64_t* uniq, hipStream_t s);
// CSR row id and local id (lid[j] = tlid[slot_of[j]]) of every non-zero;
// pos[j] = j when non-null (the sort payload of valued data)
void loc_rows_lid(const int64_t* offset, int64_t nrows, const int32_t* slot_of,
                  const int32_t* tlid, int32_t* row_of, int32_t* lid, int32_t* pos,
                  hipStream_t s);
// the CSC (per-id occurrence lists, in row order) plus per-id counts from
// lid / row_of. Scratch: pos/slid/spos [nnz] int32, sort_tmp.
size_t loc_sort_tmp_bytes(int64_t nnz, int64_t nuniq);
void loc_csc(const int32_t* row_of, const float* val, int64_t nnz, int64_t nuniq,
             int32_t* lid, int32_t* pos,
             int32_t* slid, int32_t* spos, void* sort_tmp, size_t sort_tmp_bytes,
             int64_t* csc_off, int32_t* ucnt, int32_t* csc_row, float* csc_val, hipStream_t s);

// ------------------------------------------------------ localize_part.hip
// Partitioned localize (the default path; no global atomics, no sort): a
// radix-partition pass on an owner-major digit, then one workgroup per
// partition de-duplicates, counts and places its non-zeros in LDS. Same
// outputs as the path above (uniq/ucnt/csc_off sized by an upper bound; U =
// sum of owner_cnt[0..nshard)); owner_cnt[nshard] != 0 flags a partition
// whose distinct ids overflowed its LDS table (retry on the hash path).
constexpr int kPartMaxDigits = 1024;
constexpr int kPartMaxRows = 1024;
constexpr int kPartMaxOwners = 1024;
constexpr int kPartMaxHeavy = 512;  // heavy-id partitions over all owners
struct PartPlan {
  bool ok;
  int npo_bits, nho, stride, ndig, R;  // owner o: digits [o*stride, o*stride + 2^npo_bits)
  int64_t ntiles;                      // hashed, then nho heavy-id digits
};
// Heavy-id hint: the previous minibatch's ids with >= thr occurrences, per
// owner (keys [nshard * nho], cnt [nshard]); the dedup elects this
// minibatch's into next_* (next_cnt zeroed by loc_part_hist). Any content is
// correct -- it only decides which ids get single-id partitions.
struct PartHeavy {
  const uint64_t* keys;
  const uint32_t* cnt;
  uint64_t* next_keys;
  uint32_t* next_cnt;
  int nho;       // heavy slots per owner read (0: none)
  int nho_next;  // heavy slots per owner written (0: none)
  uint32_t thr;
};
// uest: an upper estimate of the unique ids (nnz when nothing is known)
PartPlan loc_part_plan(int64_t nnz, int64_t nrows, int nshard, int64_t uest, bool heavy);
// hist [ntiles * ndig] uint32 (tile-major)
void loc_part_hist(const uint64_t* keys, const int64_t* offset, int64_t nrows, int nshard,
                   const PartPlan& pl, const PartHeavy& hv, uint32_t* hist, hipStream_t s);
// partition offsets: hist becomes the in-group tile prefix, gsum
// [loc_part_groups * ndig] the group prefix, base [ndig + 1] the digit starts
// (base[ndig] = nnz)
int64_t loc_part_groups(const PartPlan& pl);
void loc_part_offsets(const PartPlan& pl, uint32_t* hist, uint32_t* gsum, int64_t* base,
                      hipStream_t s);
// pk/pr [nnz] (+ pv [nnz] when val) in partition order; pos_of [nnz] in CSR
// order (gpre / tpre: gsum / hist after loc_part_offsets)
void loc_part_scatter(const uint64_t* keys, const float* val, const int64_t* offset,
                      int64_t nrows, int nshard, const PartPlan& pl, const PartHeavy& hv,
                      const int64_t* base, const uint32_t* gpre, const uint32_t* tpre,
                      uint64_t* pk, int32_t* pr, float* pv, int32_t* pos_of, hipStream_t s);
// up [kPartMaxDigits] u64 and *arrive (0 between calls): a workspace of its
// own; lb: a look-back workspace no concurrent kernel uses. plid [nnz]:
// local ids in partition order.
void loc_part_dedup(const uint64_t* pk, const int32_t* pr, const float* pv, int64_t nnz,
                    int nshard, const PartPlan& pl, const PartHeavy& hv, const int64_t* base,
                    const Lookback& lb,
                    uint64_t* uniq, int32_t* ucnt, int64_t* csc_off, int32_t* csc_row,
                    float* csc_val, int32_t* plid, unsigned long long* up, unsigned int* arrive,
                    int64_t* owner_cnt, hipStream_t s, int64_t* tim = nullptr);
// lid[j] = plid[pos_of[j]]
void loc_part_lid(const int32_t* pos_of, const int32_t* plid, int64_t nnz, int32_t* lid,
                  hipStream_t s);
// nnz == 0: zero owner counts and csc_off[0]
void loc_part_empty(int nshard, int64_t* owner_cnt, int64_t* csc_off, hipStream_t s);

// ---------------------------------------------------------- kvstore.hip
// Sharded parameter store (replaces the ps-lite server KVStore). Open
// addressing, linear probing, 64-bit CAS insert.
// Array-of-structs slots: every scalar of a key (its id, w, FTRL/AdaGrad
// state, count, embedding row) sits in ONE 32-byte sector, so find, pull and
// push each cost one random HBM sector per key instead of one per field.
struct alignas(32) KVSlot {
  uint64_t key;    // ~0 == empty
  float w;
  float z;         // FTRL z (linear sign convention per app)
  float sq;        // sqrt of cumulative squared gradient
  int32_t vrow;    // row into the V slab, -1 = no embedding
  uint32_t cnt;    // feature count (difacto)
  uint32_t tag;    // multi-shard open: duplicate-chain tag {epoch, index}
                   // (psx.hip); cnt and tag share one 8-byte word so the
                   // open updates both with one 64-bit atomic
};
static_assert(sizeof(KVSlot) == 32, "KVSlot must be one 32-byte sector");
// Event counters are sharded over 64 cache lines: one counter word takes
// ~12 ns per same-address atomic, and a kernel over 515K keys issues one per
// wave (8K waves -> ~100 us serialised); sharded, the adds run in parallel.
constexpr int kStatShards = 64, kStatStride = 16, kStatCount = 8;
struct KVTable {
  KVSlot* sl;         // [cap]
  float* V;           // [vcap * vstride]
  float* VG;          // [vcap * vstride] AdaGrad accumulators of V
  int32_t* vnext;     // [1] bump allocator for V rows
  int64_t* stats;     // [kStatShards][kStatStride]  0:new_w 1:new_V 2:insert_fail
                      //   3:vslab_full 4:n_keys (sum the shards to read)
  int64_t cap;        // power of two
  int64_t vcap;
  int vstride;        // padded embedding stride (multiple of 4), 0 = linear
  int dim;            // logical embedding dim
};
// find (insert=0) or find-or-insert (insert=1) each key; slot=-1 when absent
void kv_find(const KVTable& t, const uint64_t* keys, int64_t n, int insert, int32_t* slot,
             hipStream_t s);
// dump: indices of occupied slots (compaction); out_n[0] receives the count
void kv_occupied(const KVTable& t, int32_t* out_slots, int64_t* out_n, hipStream_t s);
// growth: re-insert the occupied slots of `old` into the empty table `nt`
// (power-of-two newcap > oldcap); remap[oldcap] receives old -> new slot ids
void kv_rehash(const KVSlot* old, int64_t oldcap, KVSlot* nt, int64_t newcap, int32_t* remap,
               int64_t* stats, hipStream_t s);
// health read: out[4] = {keys, failed inserts, V-slab overflows, V rows used}
void kv_summary(const KVTable& t, int64_t* out, hipStream_t s);

// ------------------------------------------------------------ linear optim
// algo: 1 SGD, 2 AdaGrad, 3 FTRL (reference learn/linear/async_sgd.h:71-180)
struct LinearHP {
  int algo;
  float alpha, beta, l1, l2;
  float sgd_eta;  // SGD only: (beta + sqrt(t)) / alpha for this push
};
void linear_pull(const KVTable& t, const int32_t* slot, int64_t n, float* out, hipStream_t s);
void linear_push(const KVTable& t, const int32_t* slot, const float* grad, int64_t n,
                 LinearHP hp, hipStream_t s);

// ----------------------------------------------------------- difacto optim
struct DifactoHP {
  float alpha, beta, l1, l2;       // FTRL on w
  float v_alpha, v_beta, v_l2;     // AdaGrad on V
  float v_init;                    // V ~ U[-v_init, v_init]
  uint32_t threshold;              // allocate V once cnt > threshold
  int l1_shrk;
  uint64_t seed;
};
// add feature counts (reference AdaGradHandle::Push with kPushFeaCnt)
// (counts as float cnt OR int32 cnti; the other is null)
void difacto_push_cnt(const KVTable& t, const int32_t* slot, const float* cnt,
                      const int32_t* cnti, int64_t n, DifactoHP hp, hipStream_t s);
// Variable-length pull (reference ZVPull, learn/difacto/async_sgd.h:234-244):
//   pass 1 (difacto_pull_hdr): hdr[i] = {w, -}, vflag[i] = key has a V row
//          (and, with l1_shrk, w != 0)
//   caller: vpos = exclusive scan of vflag (scan_i32), m = vpos[n]
//   pass 2 (difacto_pull_rows): hdr[i].y = bit-cast vpos[i] (or -1) and
//          vc[vpos[i]] = V row
void difacto_pull_hdr(const KVTable& t, const int32_t* slot, int64_t n, int l1_shrk, float* hdr,
                      int32_t* vflag, hipStream_t s);
void difacto_pull_rows(const KVTable& t, const int32_t* slot, int64_t n, const int32_t* vflag,
                       const int64_t* vpos, float* hdr, float* vc, hipStream_t s);
// push: gw[i] for every key (FTRL on w), gvc[vidx_i] for keys whose pull
// header (owner numbering) carried a V row (AdaGrad on V)
void difacto_push(const KVTable& t, const int32_t* slot, const float* hdr, const float* gw,
                  const float* gvc, int64_t n, DifactoHP hp, hipStream_t s);
// worker side of a multi-shard pull: renumber hdr[i].y into the local
// compact order (exclusive scan of hdr[i].y >= 0); tmp = n int32 +
// scan_tmp_elems(n) int64; count[0] = m
void vidx_renumber(float* hdr, int64_t n, int32_t* flag_tmp, int64_t* pos_tmp, int64_t* scan_tmp,
                   hipStream_t s);
// single-launch versions (return false when n is beyond the look-back tile
// limit; the caller then uses the multi-launch path above). The fused pull
// writes hdr {w, vidx}, vpos[n + 1] (exclusive scan of the V flags, vpos[n]
// = m) and the V rows.
bool difacto_pull_fused(const KVTable& t, const int32_t* slot, int64_t n, int l1_shrk,
                        const Lookback& lb, float* hdr, int64_t* vpos, float* vc, hipStream_t s);
// single-shard minibatch open: find-or-insert the (distinct) keys -> slot,
// add cnt (int32, may be null) with lazy V allocation, then the fused pull
bool difacto_open_pull(const KVTable& t, const uint64_t* keys, int64_t n, const int32_t* cnt,
                       DifactoHP hp, int insert, const Lookback& lb, int32_t* slot, float* hdr,
                       int64_t* vpos, float* vc, hipStream_t s);
bool vidx_renumber_fused(float* hdr, int64_t n, const Lookback& lb, int64_t* count,
                         hipStream_t s);

// ------------------------------------------------------------- psx.hip
// Multi-shard DiFacto exchange (see psx.hip for the row-aligned region
// layout). seg tables are device int64 [P+1] prefix sums: segS = key
// segment starts, segHS = header-row starts (H_p = ceil(2 n_p / vstride)).
// ps_open: owner find/insert + (use_cnt) atomic count push with lazy V
//   allocation + variable-length pull of n received keys (u64 keys, or
//   12-byte {lo, hi, count} records), writing slot/w_out/vpos[n+1], the
//   duplicate chains (chains != 0; epoch 1..255) and the reply buffer rbuf
//   (embedding rows and packed headers); vcnt[P] = V rows per peer.
//   vbase: device int32 copy of vnext taken before the launch.
// ps_push: owner applies the received push buffer (same layout as rbuf).
// ps_unpack / ps_pack_gw: worker side (segments = keys sent per owner,
//   vrecv[P] = V rows received per owner).
// Each returns false when its limits are exceeded (P > 256, n >= 2^24).
// PsPrep: the next open's preparation done by a push kernel that runs
// right before it on the same stream (zero chain[n], *vbase = vnext at the
// push's start); an open given prepped != 0 then skips its own prep launch.
struct PsPrep {
  uint32_t* chain = nullptr;
  int64_t n = 0;
  int32_t* vbase = nullptr;
};
bool ps_open(const KVTable& t, const uint64_t* keys, const int32_t* rec, int64_t n, int use_cnt,
             DifactoHP hp, int insert, int chains, uint32_t epoch, int32_t* vbase,
             const int64_t* segS, const int64_t* segHS, int P, const Lookback& lb, int32_t* slot,
             float* w_out, int64_t* vpos, uint32_t* chain, uint8_t* head, float* rbuf,
             int64_t* vcnt, hipStream_t s, int prepped = 0);
bool ps_push(const KVTable& t, const int32_t* slot, const int64_t* vpos, const uint32_t* chain,
             const uint8_t* head, int64_t n, const int64_t* segS, const int64_t* segHS, int P,
             const float* gbuf, DifactoHP hp, hipStream_t s, PsPrep prep = PsPrep());
// worker: 12-byte {lo, hi, count} records of the key exchange (ucnt may be null)
void ps_records(const uint64_t* uniq, const int32_t* ucnt, int64_t U, int32_t* rec,
                hipStream_t s);
// C0 count exchange buffers: send[4P] and payload[S+1+5P] (see psx.hip)
// loop: also fill the payload's receive slot with send (the loopback
// identity exchange, no collective)
bool ps_c0(const int64_t* owner_cnt, const int64_t* vcnt, int S, int P, int64_t flag,
           int64_t* send, int64_t* payload, hipStream_t s, int loop = 0);
// linear model (vstride 0) owner push over all P segments: chain heads apply
// their key's gradients in peer order; SGD request counter starts at t0
bool ps_push_linear(const KVTable& t, const int32_t* slot, const uint32_t* chain,
                    const uint8_t* head, int64_t n, const int64_t* segS, int P, const float* g,
                    LinearHP hp, double t0, hipStream_t s, PsPrep prep = PsPrep());
bool ps_unpack(const float* rbuf, int64_t U, int vstride, const int64_t* segS,
               const int64_t* segHS, const int64_t* vrecv, int P, float* hdr, int64_t* rows_total,
               hipStream_t s);
bool ps_pack_gw(const float* gw, int64_t U, int vstride, const int64_t* segS,
                const int64_t* segHS, const int64_t* vrecv, int P, float* gbuf, hipStream_t s);

// ---------------------------------------------------------------- fm.hip
// Forward of FM / linear model on a localized minibatch.
//   difacto: w_or_hdr = hdr[U] float2 {w, vidx}, vc = [m, vstride]
//   linear (vstride == 0): w_or_hdr = w[U], vc unused
//   loss: 1 square, 2 logit, 4 squared hinge
//   met[0..3] += {objv, objv_w, correct(threshold 0), n}  (double); with
//   loss | 256, met[4] += this minibatch's accuracy flipped below 0.5
//   part: scratch of fm_fwd_partials() doubles (per-block metric partials)
int64_t fm_fwd_partials();
// words of the forward's arrival ticket (zeroed once; left zeroed)
int64_t fwd_ticket_words();
// linear forward with w read at w[lid * wstride] (lid < 0: no weight):
// w = &table.sl[0].w, wstride = 8 reads the weights straight from the slots
void lin_forward_strided(int64_t nrows, const int64_t* offset, const int32_t* lid,
                         const float* val, const float* w, int wstride, const float* label,
                         int loss, float* py, float* dual, double* met, double* part,
                         unsigned int* ticket, hipStream_t s);
// ------------------------------------------------------- linear_direct.hip
// single-shard linear step without a localize (see the file header)
int ld_rows_per_tile(int64_t nnz, int64_t nrows);
// (nnz picks the tile table size T = ld_tile_table(nnz): pass the same value
// to ld_rows_per_tile, ld_touch and ld_backward). Slot lists: tile b writes
// its first-stamped slots to tlist[b * T ..] and their count to tcnt[b];
// ovf / *ovf_cnt hold the rare slots resolved outside a tile's LDS table
// (*ovf_cnt zero on entry; ld_push reads and re-zeroes it)
int ld_tile_table(int64_t nnz);
void ld_touch(const KVTable& t, const uint64_t* keys, const int64_t* off, int64_t nrows,
              int64_t nnz, int R, uint32_t stamp, int insert, int32_t* lid, int32_t* tlist,
              unsigned int* tcnt, int32_t* ovf, unsigned int* ovf_cnt, hipStream_t s);
void ld_backward(const int32_t* lid, const float* val, const int64_t* off, int64_t nrows,
                 int64_t nnz, int R, const float* dual, float* grad, hipStream_t s);
void ld_push(const KVTable& t, int64_t ntiles, int T, const int32_t* tlist,
             const unsigned int* tcnt, const int32_t* ovf, unsigned int* ovf_cnt, float* grad,
             LinearHP hp, hipStream_t s);
// CUs the persistent FM grids leave free for concurrent RCCL kernels
void fm_set_cu_reserve(int cus);
int fm_cu_reserve();
void fm_forward(int64_t nrows, const int64_t* offset, const int32_t* lid, const float* val,
                const float* w_or_hdr, const float* vc, int vstride, const float* label, int loss,
                float* py, float* dual, float* xv, double* met, double* part,
                unsigned int* ticket, hipStream_t s);
// Backward: gw[U] for every key, gvc[m] for the keys with an embedding row
//   gw_k = sum_i dual_i x_ik
//   gV_k = sum_i dual_i x_ik xv_i - (sum_i dual_i x_ik^2) V_k
int64_t fm_bwd_chunks_bound(int64_t nuniq, int64_t nnz);
// scratch: chunk_key/chunk_beg [fm_bwd_chunks_bound], meta_v [2 x 4 fm_bwd_meta_bound]
// int32 (16-byte aligned), bucket_hist [fm_bwd_bucket_scratch] int32,
// chunk_cnt [2 nuniq], chunk_off [2 (nuniq + 1)], scan_tmp [scan_tmp_elems(nuniq)]
int64_t fm_bwd_meta_bound(int64_t nuniq, int64_t nnz);
int64_t fm_bwd_bucket_scratch();
void fm_backward(int64_t nuniq, int64_t nnz, int64_t nrows, const int64_t* csc_off,
                 const int32_t* csc_row, const float* csc_val, const float* dual, const float* xv,
                 const float* hdr, const float* vc, int vstride, float* gw, float* gvc,
                 int32_t* chunk_key, int32_t* chunk_beg, int32_t* meta_v, int32_t* bucket_hist,
                 int64_t* chunk_cnt, int64_t* chunk_off, int64_t* scan_tmp, const Lookback* lb,
                 hipStream_t s, float* det_part = nullptr, int phase = 0);
// phase: 0 = the whole backward; 1 = only the planning that needs no dual
// (chunk lists + V-chunk bucketing: CSC offsets and the pull header), so it
// can run on a side stream concurrently with the forward; 2 = the rest
// (dual / xv dependent), after phase 1 with the same scratch.
// det_part (deterministic mode, WH_DETERMINISTIC=1): scratch of
// fm_bwd_det_floats floats; hot keys' chunk partials are then summed in
// occurrence order by a second pass instead of float atomics
int64_t fm_bwd_det_floats(int64_t nuniq, int64_t nnz, int vstride);
// post-process the m (device count) V-gradient rows: clip to [-c, c] (c>0),
// dropout with prob p (p>0); sumsq (optional) receives the squared norm
void fm_grad_post(const int64_t* m, int64_t m_cap, float* gvc, int vstride, int dim, float clip,
                  float dropout, uint64_t seed, double* sumsq, hipStream_t s);
void fm_grad_scale(const int64_t* m, int64_t m_cap, float* gvc, int vstride, int dim,
                   const double* sumsq, hipStream_t s);

// --------------------------------------------------------------- spmv.hip
// y = X x over CSR (col < 0 entries skipped); y = X^T p over the CSC of localize
void spmv(int64_t nrows, const int64_t* off, const int32_t* col, const float* val, const float* x,
          float* y, hipStream_t s);
// ------------------------------------------------------------ metrics.hip
// exact per-minibatch AUC (reference BinClassEval::AUC) from predictions
// sorted ascending: area = sum over negatives of #positives ranked below.
// (py, label) pairs sorted ascending by py (rocPRIM radix sort, float keys)
size_t auc_sort_tmp_bytes(int64_t n);
void sort_by_score(const float* py, const float* label, int64_t n, float* py_sorted,
                   float* label_sorted, void* tmp, size_t tmp_bytes, hipStream_t s);
void auc_from_sorted(const float* label_sorted, int64_t n, double* out, int64_t* tmp_i64,
                     hipStream_t s);
// Sort-free exact AUC (bucketed rank-sum, see metrics.hip), accumulated into
// *auc_sum on the device. persist: auc_ws_persistent_bytes(), zero except
// the uint64 at auc_ws_lohi_offset() = ~0 (every call restores that state;
// one per device, used in stream order). scratch: auc_ws_bytes(n).
int64_t auc_ws_bytes(int64_t n);
int64_t auc_ws_persistent_bytes();
int64_t auc_ws_lohi_offset();
void auc_accumulate(const float* py, const float* label, int64_t n, void* persist, void* scratch,
                    double* auc_sum, hipStream_t s);

// ------------------------------------------------------------ synth.hip
// Criteo-1TB-shaped synthetic minibatch: 13 integer + 26 categorical fields,
// power-law value ranks per field, keys hashed as (h>>10)|(field<<54)
// (reference learn/base/criteo_parser.h:64-86), labels from a hidden
// logistic model so the learners have signal.
void synth_criteo(int64_t nrows, uint64_t seed, uint64_t step, const int64_t* card,
                  int nfield, uint64_t* keys, float* label, int64_t* offset, hipStream_t s);

// ------------------------------------------------------------ kmeans.hip
int kmeans_ks(int f);  // padded MFMA k-steps (2 features each)
// split-precision assignment (bf16 x 3 MFMA + exact fp32 re-score of the
// near-tie rows): the exact fp32 argmax for f <= 128. Xp3 / Cp3 are opaque
// packed buffers of the given byte sizes; xnorm [n] = row L2 norms; amb
// [1 + n] int32 scratch (count, then the re-scored rows).
bool kmeans_x3_supported(int f);
int64_t kmeans_x3_xp_bytes(int64_t n, int f);
int64_t kmeans_x3_cp_bytes(int k, int f);
void kmeans_pack_x3(const float* X, int64_t n, int f, void* Xp3, hipStream_t s);
void kmeans_pack_c3(const float* C, int k, int f, void* Cp3, hipStream_t s);
void kmeans_assign_x3(const void* Xp3, const float* xnorm, const float* X, int64_t n, int f,
                      const void* Cp3, const float* C, int k, int32_t* assign, float* score,
                      int32_t* amb, float* ct, hipStream_t s);  // ct: [f * k] scratch
void kmeans_pack_x(const float* X, int64_t n, int f, float* Xp, hipStream_t s);
int64_t kmeans_cp_elems(int k, int f);  // packed centroid floats
void kmeans_pack_c(const float* C, int k, int f, float* Cp, hipStream_t s);
void kmeans_assign(const float* Xp, int64_t n, int f, const float* Cp, int k, int32_t* assign,
                   float* score, hipStream_t s);
void kmeans_accum(const float* X, int64_t n, int f, const int32_t* assign, float* sums,
                  hipStream_t s);
// the same sums through a counting sort by cluster + register segment sums
// (returns false when k / f exceed its LDS / register limits: use the above)
int64_t kmeans_accum_scratch(int64_t n, int k);
// new centroids from sums [k, f + 1] (count last) and the previous C [k, f]:
// mean (previous row if empty), L2-normalised; *nempty += empty clusters
// sparse rows (CSR, int32 columns < F) against Ct [F, Kp] (the transposed
// centroids, Kp = K rounded up to 4): argmax_k x . c_k in double
void kmeans_assign_csr(const int64_t* off, const int32_t* col, const float* val, int64_t n,
                       const float* Ct, int K, int Kp, int32_t* assign, hipStream_t s);
// sums [K, F + 1] += the rows of each cluster (atomics), column F = counts
void kmeans_accum_csr(const int64_t* off, const int32_t* col, const float* val, int64_t n,
                      const int32_t* assign, int F, float* sums, hipStream_t s);
void kmeans_update(const float* sums, const float* C, int k, int f, float* out,
                   unsigned long long* nempty, hipStream_t s);
bool kmeans_accum_sorted(const float* X, int64_t n, int f, int k, const int32_t* assign,
                         float* sums, void* scratch, hipStream_t s);

// -------------------------------------------------------------- lbfgs.hip
void owlqn_dir(const float* g, const float* w, int64_t n, float l1, float* d, hipStream_t s);
// fp64 scratch the reductions below need (doubles)
int64_t owlqn_part_doubles();
// *vdot = sum d * steep after the optional sign fix
void owlqn_fix_dot(float* d, const float* steep, int64_t n, int fix, double* part, double* vdot,
                   hipStream_t s);
// nw = fix(w + alpha d); *l1sum = |nw|_1
void owlqn_step(const float* w, const float* d, int64_t n, float alpha, int fix, float* nw,
                double* part, double* l1sum, hipStream_t s);
// out[r * K + k] = <H[r], H[probe[k]]> for r < R (row stride ld, K <= 4);
// false when n / ld are not multiples of 4 or H is not 16-byte aligned
bool hist_dots(const float* H, int R, int64_t n, int64_t ld, const int32_t* probe, int K,
               double* part, double* out, hipStream_t s);
// d = sum_r coef[r] H[rows[r]] (fp32, in list order), sign-fixed against
// H[steep_row] when fix; *vdot = sum d * steep. false if nrow > 64
bool dir_fix_dot(const float* H, int64_t n, int64_t ld, const int32_t* rows, const float* coef,
                 int nrow, int steep_row, int fix, float* d, double* part, double* vdot,
                 hipStream_t s);
// out[p] (fp64, accumulated) += <H[ia[p]], H[ib[p]]>; false if R > 64 or np > 64
bool multi_dot(const float* H, int R, int64_t n, const int32_t* ia, const int32_t* ib, int np,
               double* out, hipStream_t s);

// --------------------------------------------------------------- glm.hip
// out[v] = sum over nblk blocks of part[b * stride + v], v < nv (fixed
// order; stride 0 = nv)
void sum_parts(const double* part, int nblk, int nv, double* out, hipStream_t s, int stride = 0);
// linear-model rows over the prepared split (glm.hip header): mode 0 sums[0]
// = loss; 1 also out = pred - label and sums[1] = its sum; 2 out = margin;
// 3 out = margin and sums[0] = loss.
// part: glm_fwd_blocks(nrows) * 2 doubles
int64_t glm_fwd_blocks(int64_t nrows);
void glm_fwd(int mode, int64_t nrows, const int64_t* off, const int32_t* gcol, const float* val,
             const float* w, const float* bias, float base, const float* label, int loss,
             float* out, double* part, double* sums, hipStream_t s);
// g = pred - label from margins (+ sums {loss, sum g}; part as glm_fwd)
void glm_grad_from_margin(int64_t nrows, const float* margin, const float* label, int loss,
                          float* g, double* part, double* sums, hipStream_t s);
// run-start bits of an entry stream (glm_heads_words(nnz) u64; run u starts
// at off[u]) and X^T g into grad (zeroed by the caller) at the runs' global
// indices ucol (null: the run index itself; all_atomic: several runs may
// share one index)
int64_t glm_xtg_waves(int64_t nnz);
// grad[cgid[c]] = sum_k S[rlist[k]] over k in [coff[c], coff[c + 1])
void glm_runs_reduce(int64_t ncol, const int64_t* coff, const int32_t* rlist, const float* S,
                     const int32_t* cgid, float* grad, hipStream_t s);
int64_t glm_heads_words(int64_t nnz);
void glm_heads(const int64_t* csc_off, int64_t U, uint64_t* hb, int64_t words, hipStream_t s);
void glm_xtg(int64_t nnz, const int32_t* crow, const float* cval, const uint64_t* hb,
             const int32_t* col0w, const int32_t* ucol, const float* g, float* grad,
             int all_atomic, hipStream_t s);

// -------------------------------------------------------------- gbdt.hip
void gbdt_bin(const float* X, int64_t n, int f, const float* cuts, const int32_t* cut_off,
              uint8_t* B, hipStream_t s);
size_t gbdt_hist_lds(int fcnt, int nbin);
// tasks: int32 [ntask x 5] = {node slot, fbeg, fcnt, rbeg, rend}; hist fp64 [slots x f x nbin x 2]
int64_t gbdt_hist_pstride(int max_fcnt, int nbin);
void gbdt_hist(const uint8_t* B, int f, int nbin, const int32_t* ridx, const float* gpair,
               const float* qscale, const int32_t* tasks, int ntask, const int32_t* red, int nred,
               int max_fcnt, bool dword_rows, int64_t* part, double* hist, hipStream_t s,
               const int32_t* dseg = nullptr, int chunk = 0,
               const int32_t* ntask_dev = nullptr, bool w32 = false,
               const double* sib_hf = nullptr, const int32_t* sib_sp = nullptr,
               const int32_t* sib_par = nullptr);
// sib_hf (optional): the reduce also does gbdt_sibling's work -- hist is then
// the NEXT level's [2 x slots] histograms (built child from the sums, the
// other one as parent sib_hf[sib_par[k]] - built; sib_sp as gbdt_sibling's sp)
// w32: qscale holds {2^eg, 2^eh, R} and the blocks sum <= R rows at a time in
// int32 (see k_hist)
// ntask_dev (optional): the task count of a device-built list (ntask is then
// its upper bound; the reduce entries carry exact task counts)
// ---- the level loop on the device (gbdt_grow_dev in csrc/bind/hip_ops.cc)
int gbdt_node_rec();
// heap node records [nn x gbdt_node_rec()] -> the leaf walk's tree arrays
void gbdt_heap_tree(const double* nodes, int nn, int32_t* feat, int32_t* bin, uint8_t* defl,
                    int32_t* left, int32_t* right, float* leaf, hipStream_t s);
void gbdt_dev_apply(int S, int node0, bool last, const double* so, const double* tot,
                    const int32_t* seg, const uint8_t* alive, double eta, double alpha,
                    double lambda, double mcw, double rt_eps, double* nodes, int32_t* pfeat,
                    int32_t* pbin, uint8_t* pdefl, int32_t* lcur, int32_t* rcur, uint8_t* split,
                    uint8_t* build_left, double* tot_next, int32_t* nleft, hipStream_t s);
// lcur: the split slots' left cursors after the partition (their left
// children end there; = the segment begin when no partition ran)
bool gbdt_dev_children(int S, const int32_t* seg, const uint8_t* split, const uint8_t* build_left,
                       const int32_t* lcur, const int32_t* fg, int G, int chunk,
                       int32_t* seg_next, uint8_t* alive_next, int32_t* dseg, int32_t* sp,
                       int32_t* par, int32_t* tasks, int32_t* ntask, int32_t* red,
                       hipStream_t s);
// dseg (optional) [slots x 2] device row segments: a task's {rbeg, rend} is
// then {chunk index, chunk rows} inside its slot's segment (empty past it)
// level bookkeeping of the device-resident tree grower (see gbdt.hip)
void gbdt_child_segs(const int32_t* sp, int nsplit, const int32_t* nleft, int32_t* dseg,
                     hipStream_t s);
// one-pass (order-free) partition by per-node cursors: lcur = seg_beg, rcur =
// seg_end of the split nodes on entry; nleft [nnode] out (optional). tb:
// segment begins, tbs ints apart. false: too many segments for the LDS table
// (use goleft + scan + scatter)
bool gbdt_partition_cursor(const uint8_t* B, const uint8_t* Bc, int64_t nrows, int f,
                           const int32_t* ridx, int64_t n, const int32_t* tb, int tbs,
                           const int32_t* tn, int nt, const int32_t* node_feat,
                           const int32_t* node_bin, const uint8_t* node_defl, int32_t* lcur,
                           int32_t* rcur, const int32_t* seg_beg, int nnode, int32_t* nleft,
                           int32_t* out, hipStream_t s);
void gbdt_sibling(const double* hf, const double* hs, const int32_t* sp, const int32_t* par,
                  int nsplit, int64_t per, double* out, hipStream_t s);
// position -> node id over sorted segments tiling [0, n)
void gbdt_seg_fill(const int32_t* beg, const int32_t* node, int nseg, int64_t n, int32_t* out,
                   hipStream_t s);
// Bc: optional feature-major copy of B ([f][nrows]) for the per-row gather
void gbdt_goleft(const uint8_t* B, const uint8_t* Bc, int64_t nrows, int f, const int32_t* ridx,
                 int64_t n, const int32_t* pos_node, const int32_t* node_feat,
                 const int32_t* node_bin, const uint8_t* node_defl, int32_t* left, hipStream_t s);
void gbdt_scatter(const int32_t* ridx, int64_t n, const int32_t* pos_node, const int32_t* node_feat,
                  const int32_t* seg_beg, const int32_t* nleft, const int32_t* left,
                  const int64_t* lscan, int32_t* out, hipStream_t s);
// partition flags + exclusive scan in one look-back pass: lscan int32 [n + 1]
// (false when n needs more than kLbMaxTiles tiles: use goleft + scan_i32)
void gbdt_leaf_add(const int32_t* ridx, int64_t n, const int32_t* pos_node, const float* leaf,
                   float* margin, hipStream_t s);
// best split per node over hist [S, F, nbin, 2] (double) and totals [S, 2]:
// out [S, 6] = (gain, feature, bin, default_left, G_left, H_left); cand is
// [S * F * 4] double scratch. false when nbin > 1024.
bool gbdt_split(const double* hist, const double* totals, const uint8_t* valid, int S, int F,
                int nbin, double alpha, double lambda, double mcw, double* cand, double* out,
                hipStream_t s);
// sparse (CSR) input: global bin ids (cut_off[f] + bin, -1 = unbinned),
// compact [slots][total bins][2] histograms (tasks [ntask x 3] = {slot,
// rbeg, rend}, hq: int64 scratch of the histogram's size), split search over
// the compact layout (cand: [S x F x 5] scratch; out [S x 6] as gbdt_split,
// bin local to the feature), partition flags and tree walk on CSR rows
void gbdt_bin_csr(const int32_t* fid, const float* val, int64_t nnz, int ncol, const float* cuts,
                  const int32_t* cut_off, int32_t* gbin, hipStream_t s);
void gbdt_hist_csr(const int64_t* row_off, const int32_t* gbin, const int32_t* ridx,
                   const float* gpair, const float* qscale, const int32_t* tasks, int ntask,
                   int max_rows, int64_t tb, int nslot, int64_t* hq, double* hist, hipStream_t s);
void gbdt_split_csr(const double* hist, int64_t tb, const double* totals,
                    const int32_t* cut_off, const uint8_t* fvalid, int S, int F, double alpha,
                    double lambda, double mcw, double* cand, double* out, hipStream_t s);
void gbdt_goleft_csr(const int64_t* row_off, const int32_t* fid, const int32_t* gbin,
                     const int32_t* cut_off, const int32_t* ridx, int64_t n,
                     const int32_t* pos_node, const int32_t* node_feat, const int32_t* node_bin,
                     const uint8_t* node_defl, int32_t* left, hipStream_t s);
void gbdt_predict_csr(const int64_t* row_off, const int32_t* fid, const float* val, int64_t n,
                      const int32_t* feat, const float* thr, const int32_t* left,
                      const int32_t* right, const uint8_t* defl, const float* leaf, float* margin,
                      hipStream_t s);
// training margins after a tree: margin[i] += val[leaf of row i], walking the
// pruned tree on the row's bins (B row-major [n, f])
// gradient pairs of a boosting round + {sum g, sum h, max|g|, max|h|} (fp64)
// in one launch; scratch: gbdt_gpair_scratch() doubles, the tail zeroed once
// fixed-point histogram scales {2^eg, 2^eh[, R]} from max |g|, |h| (GBTree._qscale)
void gbdt_qscale(const float* m, double nglobal, int R, float* out, hipStream_t s);
int64_t gbdt_gpair_scratch();
void gbdt_gpair(int64_t n, const float* margin, const float* label, const float* weight,
                bool logistic, float* gpair, double* scratch, double* stats, hipStream_t s);
void gbdt_leaf_walk(const uint8_t* B, int64_t n, int f, int nn, const int32_t* feat, const int32_t* bin,
                    const uint8_t* defl, const int32_t* left, const int32_t* right,
                    const float* val, float* margin, hipStream_t s, bool lds = true);
void gbdt_predict(const float* X, int64_t n, int f, const int32_t* feat, const float* thr,
                  const int32_t* left, const int32_t* right, const uint8_t* defl,
                  const float* leaf, float* margin, hipStream_t s);

// ------------------------------------------------------------- ingest.hip
// Criteo / libsvm text -> CSR minibatch on the device (keys bit-identical to
// the host parsers'). text_lines: start [nlines + 1] of the lines of
// `text` (tile_cnt [criteo_tiles], tile_off [criteo_tiles + 1], scan_tmp
// [scan_tmp_elems(text_tiles)]); criteo_fields: padded [nlines x 39] keys +
// per-line counts + labels; criteo_compact: keys [sum counts] from the
// scanned counts.
int64_t text_tiles(int64_t nbytes);
int64_t text_lines(const uint8_t* text, int64_t nbytes, int32_t* tile_cnt, int64_t* tile_off,
                     int64_t* scan_tmp, int64_t* start, hipStream_t s);
void criteo_fields(const uint8_t* text, int64_t nbytes, const int64_t* start, int64_t nlines,
                   bool train, uint64_t* padded, int32_t* cnt, float* label, hipStream_t s);
void criteo_compact(const uint64_t* padded, const int64_t* off, int64_t nlines, uint64_t* keys,
                    hipStream_t s);
// rows sel [nsel] of a CSR block gathered into a new block with offsets noff
// [nsel + 1] (val may be null)
void csr_gather(const int64_t* off, const uint64_t* keys, const float* val, const float* label,
                const int64_t* sel, int64_t nsel, const int64_t* noff, uint64_t* okeys,
                float* oval, float* olabel, hipStream_t s);
// libsvm: cnt [nlines] features per line; then keys/val [sum cnt], label,
// weight [nlines], flags [2] (zeroed by the caller: any value != 1, any weight)
int64_t libsvm_count(const uint8_t* text, int64_t nbytes, const int64_t* start, int64_t nlines,
                     int32_t* cnt, hipStream_t s);
void libsvm_fill(const uint8_t* text, int64_t nbytes, const int64_t* start, int64_t nlines,
                 const int64_t* off, uint64_t* keys, float* val, float* label, float* weight,
                 int32_t* flags, hipStream_t s);

// -------------------------------------------------------------- quant.hip
// fixed_bytes payload filter: rows of w floats <-> packed records of
// quant_record_bytes(w, nb) bytes {float scale, w signed nb-byte ints},
// unbiased stochastic rounding (nb = 1, 2 or 3)
int64_t quant_record_bytes(int w, int nb);
void quant_rows(const float* x, int64_t rows, int w, int nb, uint64_t seed, uint8_t* out,
                hipStream_t s);
void dequant_rows(const uint8_t* in, int64_t rows, int w, int nb, float* x, hipStream_t s);
// region filter of the multi-shard exchange: desc int64 [P, 6] {sf, a, vf,
// nf, sq, ha} per peer (quant.hip); rows = wire rows of R bytes in all
void qregion_pack(const float* x, const int64_t* desc, int P, int64_t rows, int W, int nb,
                  uint64_t seed, uint8_t* out, hipStream_t s);
void qregion_unpack(const uint8_t* in, const int64_t* desc, int P, int64_t rows, int W, int nb,
                    float* x, hipStream_t s);
void trunc_u8(const int32_t* c, int64_t n, uint8_t* out, hipStream_t s);

// -------------------------------------------------------------- exchange
// gather rows: out[i, :] = in[idx[i], :]   (row width in floats)
void gather_rows(const float* in, const int32_t* idx, int64_t n, int width, float* out,
                 hipStream_t s);

}  // namespace wh
