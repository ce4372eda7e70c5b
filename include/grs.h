/* grs.h — C-ABI of libgrs, the MI355X-native (gfx950) stable LSD radix sort.
 *
 * This is the drop-in boundary for the reference's hot path: the ParallelSort compute
 * controller of amdreallyfast/GpuRadixSort.  Every entry point below names the reference
 * interface it replaces (paths relative to the reference repository root).
 *
 *   reference (OpenGL 4.5 / GLSL)                         libgrs (HIP, gfx950)
 *   ---------------------------------------------------   ---------------------------------
 *   ParallelSort::ParallelSort(const OriginalDataSsbo&)    grs_create      (scratch sized once)
 *     Include/ComputeControllers/ParallelSort.h:46,
 *     Source/ComputeControllers/ParallelSort.cpp:36-145
 *   ParallelSort::Sort()                                   grs_sort / grs_sort_bits
 *     ParallelSort.h:48, ParallelSort.cpp:168-422
 *   K1 OriginalDataToIntermediateData.comp:24-52           grs_iota_u32 (idx = i) + the key
 *                                                          extraction is the caller's layout
 *   K5 SortOriginalData.comp:27-51 + copy-back             grs_gather_records
 *     (ParallelSort.cpp:300-320)
 *   verification loop ParallelSort.cpp:325-352             grs_count_inversions
 *   durations.txt timing dump ParallelSort.cpp:357-417      grs_last_timing
 *   ~SsboBase() (Source/SSBOs/SsboBase.cpp:55-59)           grs_destroy
 *
 * Conventions:
 *  - All data pointers are HIP device pointers owned by the caller; the sorter owns its
 *    scratch (ping-pong buffers, look-back status, control block), sized at create time.
 *  - Calls are asynchronous on the given stream (a hipStream_t passed as void*; NULL = the
 *    null stream).  No call synchronises except grs_last_timing and grs_count_inversions.
 *  - The sort is stable and in place from the caller's view (the result lands back in
 *    d_keys / d_vals, as ParallelSort.cpp:311-318 copies the result back).
 *  - Errors are returned, never printed: n > capacity is GRS_ECAPACITY (the reference
 *    silently corrupts memory beyond 1,048,576 items: PrefixScanBuffer.comp:36).
 *  - One sorter per stream / host thread (the reference is single-context too).
 */
#ifndef GRS_H_
#define GRS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GRS_VERSION 410 /* 4.1.0: grs_debug_msd_flags, grs_shard_chunk_plan_host, options
                           GRS_OPT_H2_PIECE, GRS_OPT_P3, GRS_OPT_X_CHUNKS and GRS_OPT_EXCHANGE = 3
                           (additions only).  4.0.0: grs_timing gained `kind` (3.x callers'
                           structs are 4 bytes shorter); guard bands + grs_debug_check_guards;
                           grs_fill_permutation; the MSD sort's scratch allocated by capacity /
                           option */

typedef enum grs_status {
  GRS_OK = 0,
  GRS_EINVAL = 1,      /* bad argument (null pointer, bad radix/bit range, ...) */
  GRS_ENOMEM = 2,      /* hipMalloc failed */
  GRS_EHIP = 3,        /* a HIP runtime call failed; see grs_last_error() */
  GRS_ECAPACITY = 4,   /* n exceeds the sorter's capacity or GRS_MAX_N per call */
  GRS_ENODEV = 5,      /* no HIP device / bad device ordinal */
  GRS_ETIMEOUT = 6,    /* a look-back spin exceeded its bound (reported by the checks) */
  GRS_ERCCL = 7        /* an RCCL call failed (multi-GPU entry points) */
} grs_status;

/* Largest item count of one device call: 2^32 - 2^16 (look-back words hold 32-bit prefixes;
 * the reference stops at 1,048,576 items, PrefixScanBuffer.comp:36). */
#define GRS_MAX_N 0xFFFF0000ull

typedef enum grs_key_type { GRS_KEY_U32 = 0, GRS_KEY_U64 = 1 } grs_key_type;

typedef struct grs_sorter grs_sorter;

/* Per-phase GPU times of the last profiled grs_sort call (hipEvents on the call's stream).
 * Replaces the reference's durations.txt (ParallelSort.cpp:357-417), which timed host
 * submission only. */
typedef struct grs_timing {
  int passes;
  float total_ms;
  float hist_ms;             /* memset of the control block + upfront histogram */
  float pass_ms[16];         /* one onesweep launch per digit */
  float copy_ms;             /* final copy for an odd pass count (0 otherwise) */
  int kind;                  /* 0: LSD passes; 1: the MSD sort (GRS_OPT_MSD): hist_ms = the top
                                byte's sampled histogram, pass_ms[0..5] = the top-byte scatter, its
                                redo (empty unless a run outgrew its region), the per-bucket
                                byte-2 histogram, the byte-2 scatter, the LDS sort of the 16-bit
                                segments, the fallback of the longer ones; 2: every LSD pass in
                                one launch (GRS_OPT_PASS = 8): pass_ms[0] = that launch */
} grs_timing;

/* Library version (GRS_VERSION) and the last error message of this host thread. */
int grs_version(void);
const char* grs_status_string(grs_status s);
const char* grs_last_error(void);

/* Create a sorter for up to `capacity` items of key type `key_type`, optionally moving a
 * uint32 payload with every key (with_u32_payload = 1: the reference's IntermediateData
 * {_data, _globalIndexOfOriginalData} pair, Include/SSBOs/IntermediateData.h:12-30).
 * radix_bits: 4 or 8 digit width, 0 = auto (8).  device: HIP device ordinal.
 * Replaces ParallelSort::ParallelSort (ParallelSort.cpp:36-145). */
grs_status grs_create(grs_sorter** out, size_t capacity, grs_key_type key_type,
                      int with_u32_payload, int radix_bits, int device);
void grs_destroy(grs_sorter* s);

/* Bytes of device scratch the sorter holds now (second buffer, look-back status, control blocks,
 * the MSD sort's scratch, and buffers other entry points grew on demand), guard bands included.
 * Per element of capacity n (E = key + payload bytes):
 *   LSD passes (radix_bits 4, u64 pairs, capacity < 48M items):  n E + ~n/1000 E
 *   + the MSD sort's scratch (8-bit digits, u32 keys / u32 pairs / u64 keys, allocated at
 *     grs_create from 48M items of capacity, or by grs_set_option(GRS_OPT_MSD, 1)):
 *     the second buffer grows to 1.125 n + 1M elements and a region buffer of 1.3 n + 4M
 *     elements joins it, ~2.45 n E in all (C4's 2^30 u32 keys: ~10.5 GB beside its 4.3 GB of
 *     keys); grs_set_option(GRS_OPT_MSD, 0) releases it (the sorter then runs the LSD passes).
 * If the MSD scratch does not fit at grs_create, the sorter is created without it. */
size_t grs_scratch_bytes(const grs_sorter* s);

/* Debug canaries: every scratch allocation of the sorter ends in a 16-KB guard band (and the
 * arrays inside one allocation -- the two status buffers, keys and payload of the second and
 * region buffers, the MSD tables -- are separated by one), filled with a pattern when allocated.
 * Synchronises the sorter's device, counts the guard words that no longer hold the pattern (a
 * kernel wrote past one of its scratch arrays), restores them, and returns the count in
 * *bad_words (0 expected).  New with respect to the reference, whose scan silently overflows
 * past 2^20 items (PrefixScanBuffer.comp:36). */
grs_status grs_debug_check_guards(grs_sorter* s, uint64_t* bad_words);

/* TEST HOOK: what the last grs_sort of this sorter did in the MSD schedule (GRS_EINVAL when it
 * took the LSD passes): flags[0] = 1 when P1 ran twice (a run outgrew its sampled region, or the
 * keys' span put the top digit above the sample's guess), flags[1] = 1 when P2 took the exact
 * path (a sampled region overflowed, or a sort too small to sample), flags[2] = the top digit's
 * shift.  Synchronises the device.  New with respect to the reference. */
grs_status grs_debug_msd_flags(grs_sorter* s, uint32_t flags[3]);

/* Ranking used by this sorter's passes: 0 = lane-ordered LDS atomics (the default; probed on
 * the device at grs_create), 1 = wave64 ballot-match fallback (probe failed, or
 * grs_set_option(GRS_OPT_RANK, 1)).  -1 for a NULL sorter. */
int grs_rank_mode(const grs_sorter* s);

/* At-scale check of the property the atomic ranking relies on (the lanes of one returning
 * ds_add wave-instruction that hit one LDS address see the old values in ascending lane
 * order), on `device`: for each of 5 digit patterns (uniform, all equal, 4 values on one bank,
 * half the lanes on one value, 16 values on one bank) and 3 counter layouts (16 / 256 / 2048
 * bins of 32-bit counters, 256 bins of 16-bit halves), `blocks` 512-thread workgroups rank
 * `items` digits per lane with returning atomics and compare every returned value with the
 * rank a ballot match computes independently.  *mismatches = the number that differ (0 on
 * MI355X).  Synchronises.  New with respect to the reference. */
grs_status grs_lds_order_check(int device, int blocks, int items, unsigned long long* mismatches);

/* Per-sorter options: they pin what the defaults choose by size (tile shape, pass kernel,
 * record layout, ranking, the sharded exchange).  Tests pin every kernel variant through them
 * and A/B measurements compare variants with them; the defaults are the measured best, and no
 * option is ever read from the environment.  Set before the sorts they should affect (a pinned
 * small tile shape may grow the look-back status buffer: GRS_ENOMEM if that fails). */
typedef enum grs_option {
  GRS_OPT_TILE = 1,          /* -1 by size (default), 0 small (256-thread) tiles, 1 big tiles */
  GRS_OPT_XL = 2,            /* -1 by size (default), 0 never, 1 XL two-round tiles wherever big
                                tiles run (8-bit digits) */
  GRS_OPT_PASS = 3,          /* 0 by size (default), 4 one tile per workgroup (grs_onesweep_v4),
                                6 persistent workgroups with next-tile prefetch (grs_onesweep_v6),
                                8 every pass in one launch of those workgroups, a grid barrier
                                between passes (grs_onesweep_fused; slower than a kernel boundary
                                per pass on MI355X, never chosen by size) */
  GRS_OPT_RECORDS = 4,       /* u32 pairs at 8-bit digits: 0 two arrays every pass, 1 8-byte
                                (key, value) records in the sorter's scratch, 2 (default) also
                                split over the caller's arrays (even n, 8-byte aligned) */
  GRS_OPT_RANK = 5,          /* 0 (default) the device probe's choice, 1 ballot-match ranking */
  GRS_OPT_SHARDED_PATH = 6,  /* grs_sort_sharded on ONE rank: 0 (default) copy + local sort,
                                1 the G-rank path (a one-GPU rehearsal of the exchange) */
  GRS_OPT_SHARDED_SEND = 7,  /* partition-first exchange: 0 (default) one region per bucket in a
                                send buffer of (G - 1) regions + n_local items, a region being the
                                even share + 25 % + 64K items (a bucket may spill into the next
                                region; a spill is detected at the count exchange and the
                                partition is redone into contiguous buckets), 1 bucket histogram
                                + contiguous buckets always, 2 test hook: regions of n / (2G)
                                items, so full buckets spill and the redo path runs */
  GRS_OPT_EXCHANGE = 8,      /* 0 by rank count (default), 1 partition-first, 2 presorted, 3
                                chunked partition-first (keys without payload: each chunk of the
                                shard crosses the links while the next is partitioned; received
                                chunk-major; not measured on more than one GPU) */
  GRS_OPT_MERGE = 9,         /* presorted exchange, receive side: 0 (default) ceil(log2 k)
                                2-way merge rounds over the k received runs, 1 one k-way merge
                                pass (sample-delimited tiles merged in LDS; slower at 8 ranks) */
  GRS_OPT_FAULT_TILE = 10,   /* TEST HOOK: -1 (default) off; v >= 0: tile v of every pass never
                                publishes its look-back tile words and spins give up after 2^12
                                polls, so the later tiles of its look-back group time out: the
                                sort's output is wrong and GRS_ETIMEOUT surfaces through
                                grs_check_error / grs_stream_check_error (the error path's test) */
  GRS_OPT_MSD = 11,          /* u32 keys, u32 keys + u32 payload, u64 keys; 8-bit digits, the
                                whole key: -1 by size (default: from 48M keys), 0 never, 1 always
                                -- the MSD-first sort (two stable scatters by the top two bytes
                                into 65536 segments, each finished in LDS by one workgroup;
                                segments too long for LDS sorted by a segmented LSD on the bits
                                below their 16-bit prefix) instead of the LSD passes.  Also
                                grs_sort_segmented's long segments: 0 keeps them on the segmented
                                LSD instead of the top-byte scatter + LDS sorts.  2 (test hook):
                                1, with the byte-2 scatter's sampled regions refused, so its exact
                                redo runs.  Memory: 0 releases the MSD sort's scratch (~1.4 n
                                elements, grs_scratch_bytes), 1 / 2 allocate it (GRS_ENOMEM if it
                                does not fit), -1 keeps it from 48M items of capacity; a change
                                synchronises the device */
  GRS_OPT_SEG_ROUTE = 12,    /* grs_sort_segmented past the LDS-sized segments: 0 (default) by
                                shape, 1 the segmented passes (top-byte scatter + LDS runs, or the
                                segmented LSD), 2 one sort of composite (segment, key) keys */
  GRS_OPT_H2_CHUNK = 13,     /* the MSD sort's byte-2 histogram: 0 (default) by size, else the
                                keys of P1's output per workgroup (a power of two, 4096..2^20;
                                A/B runs) */
  GRS_OPT_H2_PIECE = 14,     /* the same histogram's sample: 0 (default) pieces of 256 keys, else
                                the keys of a piece (a power of two, 64..4096; A/B runs) */
  GRS_OPT_P3 = 15,           /* the MSD sort's LDS segment sort, u32 keys and u32 pairs: 0
                                (default) one workgroup per segment (u32 keys at ~2^30: the low
                                halves in LDS, three workgroups a CU), 1 persistent workgroups that
                                load the next segment while storing this one (slower; A/B runs),
                                2 one workgroup per segment, whole keys in LDS (A/B runs) */
  GRS_OPT_X_CHUNKS = 16      /* chunks of the chunked exchange (GRS_OPT_EXCHANGE = 3): 0 (default)
                                4, else 1..16; the same on every rank */
} grs_option;
grs_status grs_set_option(grs_sorter* s, grs_option opt, int value);
grs_status grs_get_option(const grs_sorter* s, grs_option opt, int* value);

/* Name of the pass kernel a sort of n items launches ("grs_onesweep_v4" or, on small grids,
 * "grs_onesweep_v6"; "grs_onesweep_region" when the MSD-first schedule runs, whose phases
 * grs_timing kind 1 reports): what profiling and roofline reports attribute the pass time to. */
const char* grs_pass_kernel(const grs_sorter* s, size_t n);

/* Stable ascending sort of d_keys[0..n) in place; when the sorter was created with a
 * payload, d_vals[0..n) is permuted with its keys (d_vals may be NULL otherwise).
 * Replaces ParallelSort::Sort() (ParallelSort.cpp:168-422).
 * Asynchronous on `stream`: until the call's work has completed, the contents of d_keys /
 * d_vals are unspecified (between passes they can hold 8-byte (key, value) records).  Keys
 * and payload must be naturally aligned (GRS_EINVAL otherwise); the passes that move 8-byte
 * records on the caller's two u32 arrays run only when both are 8-byte aligned.  Calls on one
 * sorter must be ordered (one stream, or synchronised): they share its scratch. */
grs_status grs_sort(grs_sorter* s, void* d_keys, uint32_t* d_vals, size_t n, void* stream);

/* As grs_sort, restricted to key bits [begin_bit, end_bit) (the reference's fixed
 * `for bitNumber in 0..31` loop, ParallelSort.cpp:236, made a parameter). */
grs_status grs_sort_bits(grs_sorter* s, void* d_keys, uint32_t* d_vals, size_t n,
                         int begin_bit, int end_bit, void* stream);

/* Per-phase hipEvent timing of later grs_sort calls: ring = number of most recent calls
 * whose events are kept (0 = off).  Events are recorded on each call's own stream. */
grs_status grs_set_profiling(grs_sorter* s, int ring);
/* Synchronises on the last profiled call and returns its per-phase times. */
grs_status grs_last_timing(grs_sorter* s, grs_timing* out);
/* Same for the k-th most recent profiled call (k = 0: the last one; k < ring). */
grs_status grs_timing_history(grs_sorter* s, int k, grs_timing* out);
/* Synchronises the sorter's device and returns GRS_ETIMEOUT if any look-back spin of past
 * calls gave up (the error word is then cleared). */
grs_status grs_check_error(grs_sorter* s);
/* The same for the calls issued on `stream` so far: enqueues a read-back of the error word and
 * synchronises `stream` only (the documented sync point of the checked facades:
 * ParallelSort::Sort() in grs_parallel_sort.hpp, gpuradixsort_amd.ParallelSort.Sort). */
grs_status grs_stream_check_error(grs_sorter* s, void* stream);

/* Stable key-range partition for the multi-GPU exchange (gpuradixsort_amd/sharded.py):
 * bucket(key) = number of splitters <= key (splitters: host array of n_splitters <= 15
 * non-decreasing keys of the sorter's key type).  Writes the keys (and payload) to
 * d_keys_out / d_vals_out grouped by bucket, input order kept inside each bucket, and the
 * n_splitters + 1 bucket sizes to d_counts (device uint32).  New with respect to the
 * reference, which has no multi-device path. */
grs_status grs_partition(grs_sorter* s, const void* d_keys, const uint32_t* d_vals,
                         void* d_keys_out, uint32_t* d_vals_out, size_t n,
                         const void* splitters, int n_splitters, uint32_t* d_counts,
                         void* stream);

/* Same, with splitters that break ties by position: splitter b is the element (key
 * splitters[b], shard-local index thresholds[b]) and element i of this shard goes to bucket
 * #{b : splitters[b] < key_i || (splitters[b] == key_i && thresholds[b] <= i)}.  A run of
 * equal keys can then be split between buckets (balance on duplicate-heavy inputs) while every
 * bucket stays a range of the stable order. */
grs_status grs_partition_ranges(grs_sorter* s, const void* d_keys, const uint32_t* d_vals,
                                void* d_keys_out, uint32_t* d_vals_out, size_t n,
                                const void* splitters, const uint32_t* thresholds,
                                int n_splitters, uint32_t* d_counts, void* stream);

/* The same partition into REGIONS instead of back-to-back buckets (the multi-GPU exchange's
 * send step, grs_sort_sharded): bucket b is written from d_keys_out[b * region] on (and
 * d_vals_out), so no bucket histogram (a read of the keys) precedes the pass; the bucket sizes
 * still go to d_counts.  The output arrays hold n_splitters * region + n items: a bucket larger
 * than `region` runs on into the next region (the later buckets are then wrong) but never past
 * the arrays -- a count > region says so, and grs_partition_ranges is the fallback.  Requires
 * 0 < region and (n_splitters + 1) * region < 2^32. */
grs_status grs_partition_regions(grs_sorter* s, const void* d_keys, const uint32_t* d_vals,
                                 void* d_keys_out, uint32_t* d_vals_out, size_t n,
                                 const void* splitters, const uint32_t* thresholds,
                                 int n_splitters, size_t region, uint32_t* d_counts, void* stream);

/* ---- multi-GPU: one process per GPU, RCCL over xGMI ----
 * The reference has no multi-device path; this is BASELINE config C4's exchange.  Rank r's
 * input is the global range that follows ranks < r; on return rank r holds a contiguous,
 * sorted range of the global stable order, and the ranks' outputs concatenated in rank order
 * are the stable sort of the whole input.  Two exchanges, one stream each call:
 *  - presorted (u32 keys without payload, when out_capacity >= n_local; the default there
 *    for G <= 4 ranks, GRS_OPT_EXCHANGE = 2 forces it for more):
 *    local grs_sort of the shard into d_keys_out -> regular samples of the sorted shard ->
 *    RCCL all-gather -> on-device splitters (ties broken by global index) -> bucket bounds in
 *    the sorted shard -> each bucket encoded as 256-key blocks of bit-packed deltas (about one
 *    byte per uniform key at 8 ranks) -> all-gather of the G x 2G (keys, words) matrix -> ONE
 *    host synchronisation -> grouped ncclSend / ncclRecv of the encoded words -> decode ->
 *    2-way merge rounds of the G received runs into d_keys_out (ties: source-rank order).
 *  - partition-first (payload, u64 keys, or G > 4; GRS_OPT_EXCHANGE = 1 forces it):
 *    samples
 *    -> splitters -> grs partition pass into G buckets -> all-gather of the G x G bucket
 *    counts -> ONE host synchronisation -> grouped ncclSend / ncclRecv of keys and payload ->
 *    local grs_sort of the received run (source-rank order = global order for equal keys).
 * nccl_comm: an initialised ncclComm_t (any RCCL communicator of G <= 16 ranks, one rank per
 * device); the sorter needs capacity >= max(n_local, *n_out) and out_capacity >= *n_out
 * (GRS_ECAPACITY otherwise, detected before any data moves).  Returns after enqueuing the last
 * step (check it with grs_stream_check_error); look-back timeouts before the host
 * synchronisation are reported by the call itself. */
grs_status grs_sort_sharded(grs_sorter* s, const void* d_keys_in, const uint32_t* d_vals_in,
                            size_t n_local, void* d_keys_out, uint32_t* d_vals_out,
                            size_t out_capacity, size_t* n_out, void* nccl_comm, void* stream);

/* Phases of the last multi-rank grs_sort_sharded call on this sorter (needs grs_set_profiling
 * > 0; synchronises): before_ms = samples .. the host synchronisation (partition-first: the
 * partition; presorted: local sort + encode), exchange_ms = the grouped send / recv and the self
 * copy, after_ms = local sort (partition-first) or decode + merge (presorted).  bytes_* count
 * what crossed the links (the self part excluded); bytes_sent / exchange_ms is the xGMI rate
 * of this rank. */
typedef struct grs_sharded_timing {
  float total_ms, before_ms, exchange_ms, after_ms;
  uint64_t bytes_sent, bytes_received;
  int presorted;
} grs_sharded_timing;
grs_status grs_sharded_last_timing(grs_sorter* s, grs_sharded_timing* out);
/* Partition-first calls whose region send buffer overflowed (a bucket larger than its region)
 * and were redone into contiguous buckets, since the sorter was created. */
grs_status grs_sharded_redo_count(const grs_sorter* s, uint64_t* count);

/* RCCL communicator helpers for callers without their own RCCL binding (ctypes, tests):
 * rank 0 creates the id (GRS_RCCL_ID_BYTES bytes), every rank passes it to comm_init. */
#define GRS_RCCL_ID_BYTES 128
grs_status grs_rccl_unique_id(void* id_out);
grs_status grs_rccl_comm_init(void** comm_out, const void* id, int nranks, int rank, int device);
void grs_rccl_comm_destroy(void* comm);

/* Host twins of the sharded sort's host-visible arithmetic (no device needed; the CPU tests
 * run the orchestration under gloo with them):
 *  - splitters of `rank` from the G*S gathered samples sorted by (key, gathered index):
 *    sorted_keys / sorted_idx (M = G*S entries), gathered_pos (shard position of sample j);
 *    writes G-1 splitter keys and this rank's thresholds (the device step's exact output).
 *  - the exchange plan from the G x G count matrix (row r = what rank r sends to each bucket):
 *    send / receive offsets per peer and the received total. */
grs_status grs_shard_splitters_host(const void* sorted_keys, const uint32_t* sorted_idx,
                                    const uint32_t* gathered_pos, int key_bytes, int nranks,
                                    int samples_per_rank, int rank, void* splitters_out,
                                    uint32_t* thresholds_out);
grs_status grs_shard_plan_host(const uint32_t* count_matrix, int nranks, int rank,
                               uint64_t* send_off, uint64_t* recv_off, uint64_t* n_out);
/* The presorted exchange's bucket bounds in a SORTED shard (the device step grs_shard_bounds):
 * bounds_out[0] = 0, bounds_out[G] = n, bounds_out[b+1] = clamp(thresholds[b], lower_bound,
 * upper_bound of splitters[b]); bucket b = [bounds_out[b], bounds_out[b+1]). */
grs_status grs_shard_bounds_host(const void* sorted_keys, size_t n, int key_bytes,
                                 const void* splitters, const uint32_t* thresholds, int nranks,
                                 uint64_t* bounds_out);
/* The chunked exchange's plan (GRS_OPT_EXCHANGE = 3): count_matrices = nchunks G x G matrices
 * (chunk c's row r = what rank r's chunk c sends to each bucket; chunk c of a shard starts at
 * c * chunk_len, its buckets contiguous from there in the send buffer).  Received chunk-major:
 * send_off / recv_off get nchunks x G offsets, n_out the received total. */
grs_status grs_shard_chunk_plan_host(const uint32_t* count_matrices, int nchunks, int nranks, int rank,
                                     uint64_t chunk_len, uint64_t* send_off, uint64_t* recv_off,
                                     uint64_t* n_out);
/* Samples per rank of the sharded sort for nranks ranks (min(1024, 8192 / nranks)). */
int grs_shard_samples_per_rank(int nranks);

/* The presorted exchange as transport-independent steps (u32 keys, no payload), for hosts
 * that move the bytes themselves (MPI, gloo, a simulated exchange on one device).  Rank r:
 *   1. sort its shard (grs_sort);
 *   2. grs_shard_sample: S = grs_shard_samples_per_rank(G) samples of the SORTED shard;
 *      all-gather them rank-major (keys and positions, G*S each);
 *   3. grs_shard_encode: splitters, bucket bounds, encoding; d_send gets the G buckets back to
 *      back (d_send_capacity_words >= grs_shard_encode_words_max(n, G)); d_sizes (device, 2G
 *      u32) gets bucket b's key count [2b] and encoded words [2b+1];
 *   4. all-gather the sizes; send bucket p's words to rank p, receive source p's words;
 *   5. grs_shard_decode_merge: recv_word_offsets[p] / recv_keys[p] (host arrays) locate source
 *      p's words in d_recv and its key count; writes the merged range to d_keys_out.
 * The sorter needs capacity >= the received total (its ping-pong buffer is the merge scratch). */
grs_status grs_shard_sample(const void* d_keys, size_t n, int key_bytes, int samples,
                            void* d_sample_keys, uint32_t* d_sample_pos, void* stream);
size_t grs_shard_encode_words_max(size_t n, int nranks);
grs_status grs_shard_encode(grs_sorter* s, const uint32_t* d_sorted, size_t n,
                            const uint32_t* d_gathered_keys, const uint32_t* d_gathered_pos,
                            int nranks, int rank, uint32_t* d_send, size_t send_capacity_words,
                            uint32_t* d_sizes, void* stream);
grs_status grs_shard_decode_merge(grs_sorter* s, const uint32_t* d_recv, int nranks,
                                  const uint64_t* recv_word_offsets, const uint32_t* recv_keys,
                                  uint32_t* d_keys_out, size_t out_capacity, void* stream);

/* ---- boundary helpers (reference K1/K5/verification, synthetic data) ---- */

/* d_out[i] = start + i  (K1's idx = tid, OriginalDataToIntermediateData.comp:42). */
grs_status grs_iota_u32(uint32_t* d_out, size_t n, uint32_t start, void* stream);

/* d_dst[i] = d_src[d_idx[i]] for records of record_bytes bytes (K5 gather,
 * SortOriginalData.comp:27-51; the caller then owns the sorted copy). */
grs_status grs_gather_records(const void* d_src, void* d_dst, const uint32_t* d_idx, size_t n,
                              size_t record_bytes, void* stream);

/* d_dst[i] = d_src[i] with the pass kernel's access width (one 4-byte word per lane, 256 B per
 * wave-instruction): a kernel of known bytes that calibrates rocprofv3's FETCH_SIZE /
 * WRITE_SIZE counters for the pass's loads and stores (bench.py's roofline.traffic). */
grs_status grs_copy_u32(const uint32_t* d_src, uint32_t* d_dst, size_t n, void* stream);

/* Synthetic keys of SURVEY §8(d): key[i] = splitmix64(seed ^ (first_index + i)) truncated
 * to key_bytes (4 or 8). */
grs_status grs_fill_splitmix(void* d_keys, size_t n, int key_bytes, uint64_t seed,
                             uint64_t first_index, void* stream);

/* The reference's own input, 0..total-1 shuffled (main.cpp:119-125): key[i] = pi(first_index + i)
 * for a seeded bijection pi of [0, total) (four multiply-xorshift rounds on the next power of two,
 * cycle-walked below total); first_index + n <= total, total <= 2^32 for 4-byte keys.  Sharded
 * callers fill rank r's slice with first_index = r * n_local. */
grs_status grs_fill_permutation(void* d_keys, size_t n, int key_bytes, uint64_t total, uint64_t seed,
                                uint64_t first_index, void* stream);

/* Number of i in [1, n) with key[i] < key[i-1] (the reference's monotonic check,
 * ParallelSort.cpp:336-352).  Synchronises. */
grs_status grs_count_inversions(const void* d_keys, size_t n, int key_bytes,
                                uint64_t* out_count, void* stream);

/* Host-buffer sort (BASELINE config C1's plumbing path; the reference's glBufferSubData
 * upload + Sort() + readback, main.cpp:146-160): copies h_keys_in (and h_vals_in) to device
 * staging owned by the sorter, sorts, copies the result to h_keys_out (and h_vals_out), and
 * synchronises `stream`.  In-place (h_keys_out == h_keys_in) is allowed.  Its rate includes
 * PCIe both ways; bench.py's headline value never does. */
grs_status grs_sort_host(grs_sorter* s, const void* h_keys_in, void* h_keys_out,
                         const uint32_t* h_vals_in, uint32_t* h_vals_out, size_t n, void* stream);

/* ---- beyond the reference's path ---- */

/* Order-preserving key transforms, so that signed and floating-point keys sort with the
 * unsigned radix sort (the reference sorts unsigned keys only, ReadMeRadixSort.txt:71-80;
 * its K1 key hook is OriginalDataToIntermediateData.comp:12-19,42).  kind: 0 unsigned
 * (no-op), 1 two's-complement signed, 2 IEEE-754 (f32 / f64; -NaN < -inf < -0 < +0 < +inf <
 * +NaN).  inverse = 0 before the sort, 1 after it.  In place, asynchronous. */
#define GRS_KEYS_UNSIGNED 0
#define GRS_KEYS_SIGNED 1
#define GRS_KEYS_FLOAT 2
grs_status grs_key_transform(void* d_keys, size_t n, int key_bytes, int kind, int inverse,
                             void* stream);

/* Record sort with a key-extraction hook: the reference's K1 (OriginalDataToIntermediateData
 * .comp:12-19,42: "adapt to whatever needs to be sorted") + pair sort + K5 gather + copy-back
 * (SortOriginalData.comp:27-51, ParallelSort.cpp:300-320), for records of any size — the use
 * the reference is built for: "sort the particles ... by Morton codes" (ParallelSort.h:13-31).
 * One fused pre-pass extracts every record's key (and its index), the (key, index) pairs are
 * sorted stably, the records are gathered by index into sorter-owned scratch and copied back,
 * so d_records[0..n) ends up sorted in place.  Needs a sorter created with a payload; the key
 * width is the sorter's (u32 / u64).
 *   GRS_EXTRACT_FIELD    key = the key-width field at byte `offset` of the record, through
 *                        `transform` (GRS_KEYS_UNSIGNED / SIGNED / FLOAT: signed and IEEE
 *                        fields sort in their own order)
 *   GRS_EXTRACT_MORTON3  key = Morton (Z-order) code of the float x, y, z at `offset`,
 *                        offset + 4, offset + 8: each axis mapped to [0, 2^B) by
 *                        floor((v - lo) / (hi - lo) * 2^B), clamped (NaN -> 0), B = 10 for
 *                        u32 keys, 21 for u64; bits interleaved x-y-z from the top
 * Scratch (keys + index + one copy of the records) is sized for the call, grown on demand and
 * kept. */
#define GRS_EXTRACT_FIELD 0
#define GRS_EXTRACT_MORTON3 1
typedef struct grs_key_extract {
  int kind;           /* GRS_EXTRACT_* */
  uint32_t offset;    /* byte offset of the field (FIELD) or of x (MORTON3) in the record */
  int transform;      /* FIELD: GRS_KEYS_UNSIGNED / SIGNED / FLOAT */
  float lo[3];        /* MORTON3: lower bounds of x, y, z */
  float hi[3];        /* MORTON3: upper bounds of x, y, z */
} grs_key_extract;
grs_status grs_sort_records(grs_sorter* s, void* d_records, size_t n, size_t record_bytes,
                            const grs_key_extract* key, void* stream);

/* The same record sort with a caller-defined key (the reference's K1 is "adapted to whatever
 * needs to be sorted", OriginalDataToIntermediateData.comp:12-19): the caller's own kernel has
 * written d_keys[i] = key of record i (the sorter's key width) and d_idx[i] = i, stream-ordered
 * before this call; the (key, index) pairs are sorted stably (both buffers are overwritten),
 * the records gathered by index and copied back, so d_records[0..n) ends up sorted in place.
 * grs_records_key_buffers hands out sorter-owned device buffers for the keys and indices,
 * laid out for the sorter's capacity (any n <= capacity may be sorted with them; their own
 * allocation, made on first use); they stay valid until grs_destroy.  The record copy of a
 * call is a separate buffer sized for that call's n and record size.  The C++ template
 * grs::ParallelSortBy (grs_parallel_sort.hpp) wraps both around a __device__ key functor. */
grs_status grs_records_key_buffers(grs_sorter* s, size_t n, size_t record_bytes, void** d_keys,
                                   uint32_t** d_idx);
grs_status grs_sort_records_by_keys(grs_sorter* s, void* d_records, size_t n, size_t record_bytes,
                                    void* d_keys, uint32_t* d_idx, void* stream);

/* Stand-alone device-wide exclusive prefix sum of uint32 (sums wrap mod 2^32), the
 * reference's K3a + K3b (ParallelPrefixScan.comp:41-196, ParallelSort.cpp:253-274) in one
 * pass with a decoupled look-back (8 B of HBM traffic per item).  d_out may equal d_in; both
 * 16-byte aligned.
 * d_total (nullable) receives the sum of all items (the reference's totalNumberOfOnes,
 * PrefixScanBuffer.comp:37).  Scratch: device memory of grs_scan_scratch_bytes(n) bytes,
 * 8-byte aligned, owned by the caller, one call at a time. */
#define GRS_SCAN_MAX_N 0xFFFFF000u
size_t grs_scan_scratch_bytes(size_t n);
grs_status grs_exclusive_scan_u32(const uint32_t* d_in, uint32_t* d_out, size_t n,
                                  uint32_t* d_total, void* d_scratch, size_t scratch_bytes,
                                  void* stream);
/* Synchronises on `stream`; GRS_ETIMEOUT if the last scan's look-back spin gave up. */
grs_status grs_scan_check_error(const void* d_scratch, void* stream);

/* Segmented (batched) stable sort: every segment [off[s], off[s+1]) of d_keys[0..n) is
 * sorted on its own, with d_vals (nullable) permuted alike; d_offsets: num_segments + 1
 * non-decreasing DEVICE words, off[0] = 0, off[num_segments] = n.  Needs a sorter created
 * with a payload.  Where no segment is longer than 16384 items (u32 keys; 8192 for u64 keys,
 * 4096 where the LDS lane-order probe failed), one workgroup per segment sorts it in LDS (one
 * read and one write of the data); finding the longest segment costs one synchronisation of
 * `stream` (skipped when the average segment is already longer).  Otherwise, with at most 16
 * segments, each segment is sorted on its own (the offsets are read back: one synchronisation);
 * with more, two sorts (keys, then segment ids; for u32 keys one sort of (segment, key)) and a
 * gather; scratch of 12 + key-size bytes per item is allocated on first use and kept. */
grs_status grs_sort_segmented(grs_sorter* s, void* d_keys, uint32_t* d_vals, size_t n,
                              const uint32_t* d_offsets, int num_segments, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GRS_H_ */
