/*
 * kstep_fmi.h -- C ABI of the MI355X k-step FM-index backward-search engine
 * (libkstepfmi.so, built from k-step_fm-index_amd/).
 *
 * Section 1 is the reference's own link-time plugin interface
 * (/root/reference/common/interface.h:27-41) plus the common.h helpers its
 * driver calls (/root/reference/common/common.h:87-96): a program written
 * against the reference (common/searchQueries.c) links against this library
 * instead of common.c + fmIndexCPUBaseline*.c + one fmIndexGPU-*.cu file, and
 * runs unchanged.  All handles are opaque `void *`; every
 * size that can exceed 2^32 bytes is 64-bit internally (reference defect B7).
 *
 * Section 2 holds the extensions that the reference fixes at compile time
 * (backend, device, K, d) or does not have (memory-resident handles, status
 * queries, timing, the GPU index builder).  Plain C types only.
 *
 * Error codes are the reference's error_t (common.h:36-62); the index-tag
 * codes 100/101/200/201 mean "this backend needs an index with that tag".
 */
#ifndef KSTEP_FMI_H_
#define KSTEP_FMI_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error_t values, common.h:36-62 */
enum {
  KFMI_SUCCESS                = 0,
  KFMI_E_OPENING_INDEX_FILE   = 1,
  KFMI_E_ALLOCATING_BWT       = 2,
  KFMI_E_ALLOCATING_FMI       = 3,
  KFMI_E_READING_BWT          = 4,
  KFMI_E_READING_FMI          = 5,
  KFMI_E_SAVING_INDEX_FILE    = 6,
  KFMI_E_SAVING_BWT_FILE      = 7,
  KFMI_E_BUILDING_BWT         = 8,
  KFMI_E_BUILDING_FMI         = 9,
  KFMI_E_OPENING_REFERENCE_FILE = 10,
  KFMI_E_ALLOCATING_REFERENCE = 11,
  KFMI_E_READING_MFASTA_FILE  = 12,
  KFMI_E_READING_REFERENCE_FILE = 13,
  KFMI_E_OPENING_MFASTA_FILE  = 14,
  KFMI_E_ALLOCATING_MFASTA    = 15,
  KFMI_E_ALLOCATING_RESULTS   = 16,
  KFMI_E_OPENING_RESULTS_FILE = 17,
  KFMI_E_READING_RESULTS_FILE = 18,
  KFMI_E_NOT_IMPLEMENTED      = 19,
  /* extensions (not in the reference) */
  KFMI_E_NO_DEVICE            = 30,  /* no HIP device / HIP runtime error      */
  KFMI_E_DEVICE_ALLOC         = 31,  /* hipMalloc failed                        */
  KFMI_E_KERNEL               = 32,  /* kernel launch / execution failed        */
  KFMI_E_BAD_ARGUMENT         = 33,  /* unsupported K, d, query size, backend   */
  KFMI_E_NOT_ON_DEVICE        = 34,  /* search called before transferCPUtoGPU   */
  KFMI_INDEX_VER_BASELINE      = 100,
  KFMI_INDEX_VER_INTERLEAVE    = 101,
  KFMI_INDEX_VER_BASELINE_AC   = 200,
  KFMI_INDEX_VER_INTERLEAVE_AC = 201
};

/* ===================== 1. reference entry points ======================== */

/* interface.h:27 / fmIndexCPUBaseline.c:71-143.  Reads any index tag
 * (100/101/200/201).  With KFMI_STRICT_TAG=1 in the environment it behaves
 * exactly like the reference loader of the selected backend: a file with
 * another tag is rejected and the required tag is returned. */
int32_t loadIndex(const char *fn, void **index);
/* interface.h:28 / genFMindex.c:155-181: "<fn>.<n>.<d>fmi<K>steps.fmi" (tag 100),
 * or the index's own tag/name suffix for transformed indexes. */
int32_t saveIndex(const char *fn, void *index);
/* interface.h:29 / common.c:248-260: 2*numresults u32, zeroed. */
int32_t initResults(uint32_t numresults, void **results);
/* interface.h:31 / fmIndexGPU-*.cu searchIndexGPU: synchronous search of every
 * query on the device; results stay on the device until transferGPUtoCPU.
 * Returns void like the reference; kfmi_last_error() gives the status. */
void    searchIndexGPU(void *index, void *queries, void *resIntervals);
/* interface.h:30 / fmIndexCPUBaseline.c:157-292 (tags 100/101) and
 * fmIndexCPUBaseline-AltCounters.c:145-310 (tags 200/201): the search on the
 * host, same integers as the reference's CPU searchers.  Like the reference it
 * is called by every thread of the caller's OpenMP parallel region
 * (searchQueries.c:84-95) and shares the queries out with an orphaned
 * `omp for schedule(static)` (GNU OpenMP); called outside a parallel region it
 * runs on the calling thread.  Results go to the host results array; a later
 * saveResults writes "<fn>.res.cpu" as the reference's CPU build does.
 * Returns void like the reference; kfmi_last_error() gives the status (33:
 * unsupported index or query size -- AltCounters indexes need m % K == 0). */
void    searchIndexCPU(void *index, void *queries, void *resIntervals);
/* interface.h:33 / fmIndexCPUBaseline.c:145-155 */
int32_t freeIndex(void **index);
/* interface.h:34 / common.c:313-322 */
int32_t freeReference(void **reference, void **index);
/* interface.h:35 / genFMindex.c:457-543: tag-100 index of a loadRef() text,
 * K and d from KFMI_K / KFMI_D (defaults 2 / 64); built on the GPU when one
 * is present (kfmi_build_index_gpu), else on the host. */
int32_t buildIndex(void *reference, void **index);
/* interface.h:36-41 / e.g. fmIndexGPU-Coop-2Step.cu:231-338 */
int32_t freeQueriesGPU(void **queries);
int32_t freeResultsGPU(void **results);
int32_t freeIndexGPU(void **index);
int32_t transferGPUtoCPU(void *results);
/* The reads go up as ASCII (the reference's form); KFMI_UPLOAD=packed (K in
 * {1, 2, 4}) packs them to 2-bit code words on the host during the upload
 * instead -- a quarter of the PCIe bytes, a win where the host workers
 * out-pack the link; same results. */
int32_t transferCPUtoGPU(void *index, void *queries, void *results);
/* How transferCPUtoGPU left the reads: 0 not on a device, 1 ASCII, 2 code
 * words packed by the host (a device group: its first member's slice). */
int32_t kfmi_queries_upload_form(void *queries);

/* common.h:87-96 / common.c */
double   sampleTime(void);
uint32_t base2index(uint32_t base);
int32_t  loadRef(const char *fn, uint32_t refsize, void **reference);
int32_t  saveRef(const char *fn, void *reference);
int32_t  loadQueries(const char *fn, uint32_t sizequery, uint32_t numqueries, void **queries);
int32_t  writeResults(const char *fn, uint32_t *results, uint32_t numqueries);
int32_t  loadResults(const char *fn, void **results);
int32_t  freeQueries(void **queries);
int32_t  freeResults(void **results);
/* common.c:324-341: "<fn>.res.gpu", or "<fn>.res.cpu" when searchIndexCPU wrote
 * the results last (the reference names the file by its build, CUDA or not) */
int32_t  saveResults(const char *fn, void *results, void *index);
char    *errorCommon(int32_t e);

/* ========================= 2. extensions ================================= */

/* Backends (the reference selects one per binary at link time,
 * makefile:177-207).  Names:
 *   "task"        Task-{1,2}Step   : one thread per query, L and R ends      (tag 101 semantics)
 *   "coop"        Coop-{1,2}Step   : wave64 cooperative gather into LDS     (tag 101 semantics)
 *   "task-ac"     Task-2Step-AltCounters                                    (tag 201 semantics)
 *   "coop-ac"     Coop-2Step-AltCounters                                    (tag 201 semantics)
 *   "task-mid"    task-per-query on the MID128 layout: one 128-byte line per LF (tag 101 semantics)
 *   "coop-mid"    wave64 cooperative gather on the MID128 layout              (tag 101 semantics)
 *   "task-grp" / "coop-grp"   K = 3 and 4 indexes (d = 64): one 128-byte line per (block,
 *                 16-code group) holding the block's planes and those 16 counters -- one line per
 *                 LF, 25 K-steps for 100 bases at K = 4; 4 (K = 3) or 16 (K = 4) lines per block
 *                 (tag 101 semantics)
 *   "task-ac-mid" / "coop-ac-mid" the MID128 lines with AltCounters semantics: the AltCounters
 *                 step only past the last real block, from the tfmiAC sentinel (tag 201 semantics;
 *                 built from a tag 100/101 file, an AC file returns 101)
 * ("task-packed" / "coop-packed" and "task-ac128" / "coop-ac128", layouts that
 * lost to task-mid / task-ac on every measurement, were retired in round 6:
 * kfmi_set_backend returns KFMI_E_BAD_ARGUMENT for them.)
 * The default comes from KFMI_BACKEND, else "task-mid" -- and "coop-grp" for a
 * K = 3 or 4 index while neither KFMI_BACKEND nor kfmi_set_backend has chosen one
 * (kfmi_get_backend still names the selection).  transferCPUtoGPU
 * re-lays-out the loaded index for the backend: plain-counter backends take
 * tag 100 or 101 (an AC file returns 101, as the reference loader would);
 * AC backends take any tag -- a tag-100/101 file first goes through the tfmiAC
 * transform, so the results are those of the AltCounters searcher on it. */
int32_t     kfmi_set_backend(const char *name);
const char *kfmi_get_backend(void);
/* The HIP device used by the calling thread (reference: compile-time DEVICE).
 * Default: KFMI_DEVICE, else 0. */
int32_t     kfmi_set_device(int32_t device);
int32_t     kfmi_device_count(void);
/* PCI bus id ("0000:75:00.0") of HIP device `device`, NUL-terminated in buf
 * (len >= 13): names the physical GPU, which device numbers do not across
 * processes with different HIP_VISIBLE_DEVICES (not in the reference, which
 * has one compile-time DEVICE). */
int32_t     kfmi_device_pci_bus_id(int32_t device, char *buf, int32_t len);
/* Status of the last searchIndexGPU() on this thread. */
int32_t     kfmi_last_error(void);
/* searchIndexGPU with a status return. */
int32_t     kfmi_search(void *index, void *queries, void *results);
/* searchIndexCPU in a parallel region of its own: nthreads threads (0:
 * OMP_NUM_THREADS when set, else this process's CPUs -- affinity mask capped
 * by the cgroup quota).  Returns the status. */
int32_t     kfmi_search_cpu(void *index, void *queries, void *results, int32_t nthreads);
/* ftab (Bowtie-style jump start; not in the reference): every backend looks
 * up [L, R) after the first `bases` bases of each query in a table of all
 * 4^bases codes (8 B each: 134 MB at 12) built on the device with the search's
 * own LF steps, then continue from there -- results are unchanged.  0 = off
 * (default; KFMI_FTAB, read once at the first search, sets it process-wide),
 * at most 16, a multiple of K to
 * take effect; per calling thread like the backend. */
int32_t     kfmi_set_ftab(uint32_t bases);
/* Test knobs of the search path (not in the reference), process-wide; their
 * environment variables are read once, at the first search, and these setters
 * switch them afterwards.  Split class (KFMI_SPLIT): the fetch form the task
 * kernels use for an index of that table-size class -- 0 = by the uploaded
 * table's size (default), 1 (< 2 GB), 2 (2-3.5 GB), 4 (larger); other values
 * KFMI_E_BAD_ARGUMENT.  Fused packing (KFMI_FUSED): 1 = reads of up to 256
 * K-step bases are packed inside the search kernel (default), 0 = always the
 * separate pack launch.  Results are identical either way. */
int32_t     kfmi_set_split_class(uint32_t cls);
int32_t     kfmi_set_fused(int32_t on);
/* Walk check of locate and the K = 2 -> 4 derivation (every LF_K walk must end
 * at a '$' row; indexes that fail are refused with KFMI_E_BUILDING_FMI), run
 * once per device copy: 0 = by size (default: full pointer jumping below 2^22
 * rows, the sampled check above), 1 = always full pointer jumping, 2 = always
 * the sampled check (which falls back to full jumping when it cannot decide);
 * other values KFMI_E_BAD_ARGUMENT.  Test knob, process-wide, no environment
 * variable.  kfmi_walk_check_last: how the last check decided -- 0 none yet,
 * 1 full, 2 sampled, 3 sampled then full. */
int32_t     kfmi_set_walk_check(uint32_t mode);
int32_t     kfmi_walk_check_last(void);
/* Every entry point leaves the caller's current HIP device as it found it
 * (hipGetDevice before == after), whichever devices it used inside. */
/* Device groups (runtime multi-GPU behind the same handles; the reference
 * picks one GPU at compile time with -DDEVICE, Coop-2Step.cu:256).  With two
 * or more devices listed -- here or in KFMI_DEVICES=0,1,... -- transferCPUtoGPU
 * replicates the index on every device and cuts queries and results into
 * contiguous slices (multiples of 64 reads), searchIndexGPU runs all slices
 * concurrently (one stream per device) and transferGPUtoCPU gathers them into
 * h_results; results equal the single-device ones.  A device may be listed
 * twice (two replicas on one GPU).  n = 0 returns to single-device mode, n = 1
 * equals kfmi_set_device.  Per calling thread.  kfmi_locate works on group
 * handles (each device locates its slice), so does kfmi_search_stream (one
 * slice and host thread per member), and reads parsed on a device
 * (kfmi_load_queries_gpu) reach the members device to device, and
 * kfmi_count_blocks sums the members' slices. */
int32_t     kfmi_set_devices(const int32_t *devices, int32_t n);
/* The device list (returns its length; 0 = single-device mode). */
int32_t     kfmi_get_devices(int32_t *devices, int32_t cap);
/* Device-side timing of the last search, from HIP events on the library's
 * stream: total (pack + LF), query packing, and the LF kernel alone (ms). */
int32_t     kfmi_last_timing(double *ms_total, double *ms_pack, double *ms_lf);

/* Strict loader: as the reference, rejects a tag other than `required_tag`
 * and returns that tag (common.c:304-307 turns it into a hint). */
int32_t kfmi_load_index_tag(const char *fn, uint32_t required_tag, void **index);
/* Index from an in-memory file image (header + entries); the bytes are copied. */
int32_t kfmi_index_from_image(const void *image, uint64_t bytes, void **index);
/* Serialised file image of an index (header + entries); pointer owned by the index. */
int32_t kfmi_index_image(void *index, const void **image, uint64_t *bytes);
/* Header fields: out[0..5] = tag, steps, bwtsize, ncounters, nentries, chunk;
 * out[6..9] dollarPositionBWT; out[10..13] dollarBaseBWT. */
int32_t kfmi_index_header(void *index, uint32_t *out14);

/* Layout transforms (transformIndexBitmaps.c:269-295, transformIndexAlternateCounters.c:387-479). */
int32_t kfmi_transform_interleave(void *index100, void **index101);
int32_t kfmi_transform_ac(void *index100, void **index200, void **index201);
/* The inverse of kfmi_transform_ac: a tag-200/201 (AltCounters) index back to
 * the tag-100 file it came from, byte for byte (no reference counterpart; the
 * AltCounters-semantics MID128 backends take AltCounters files through it). */
int32_t kfmi_transform_plain(void *index_ac, void **index100);

/* Queries/results handles over caller memory-resident data (the FFI form of
 * loadQueries/initResults).  `ascii` is num*size bytes, query q at q*size. */
int32_t   kfmi_queries_from_buffer(const char *ascii, uint64_t num, uint32_t size, void **queries);
int32_t   kfmi_results_alloc(uint64_t num, void **results);
uint32_t *kfmi_results_host(void *results);      /* 2*num u32, [L0,R0,L1,R1,...] */
uint64_t  kfmi_results_num(void *results);

/* Index construction (genFMindex.c:457-543) from an ACGT text of n bases.
 * _gpu: suffix sort and all layout passes on the device.  want_host_image != 0
 * copies the tag-100 image to host memory at once; 0 keeps the entries in HBM
 * only (the handle owns them): transferCPUtoGPU then lays them out device to
 * device, and the host image is fetched on first use (kfmi_index_image,
 * saveIndex, the transforms, the AltCounters layouts).  Returns a tag-100
 * index. */
int32_t kfmi_build_index_cpu(const char *text, uint64_t n, uint32_t k, uint32_t d, void **index);
int32_t kfmi_build_index_gpu(const char *text, uint64_t n, uint32_t k, uint32_t d,
                             int32_t want_host_image, void **index);
/* A 2K-step index derived on the current device from a K-step one (K = 1 or
 * 2, tag 100 or 101; k_out = 2K), without the text: row i's 2K-mer is its
 * K-mer plus the K-mer of row LF_K(i) (DESIGN.md 5d').  The result is the
 * tag-100 index the builders write for that text at k_out, byte for byte
 * (ACGT texts; an index with an LF_K walk that never reaches a '$' row --
 * 'ref'-mode indexes of texts with other bytes -- returns
 * KFMI_E_BUILDING_FMI, from the walk check run before deriving, see
 * kfmi_set_walk_check); its entries stay in HBM unless want_host_image.  The
 * reference's K = 2 files thus search on the K = 4 layout (coop-grp). */
int32_t kfmi_derive_index_gpu(void *index, uint32_t k_out, int32_t want_host_image, void **out);
/* Alphabet of the builders (process-wide; NULL = KFMI_ALPHABET, else "acgt"):
 *   "acgt" only A/C/G/T (anything else: KFMI_E_BUILDING_BWT);
 *   "map"  every byte through base2index (N -> G, lowercase -> uppercase), a
 *          consistent index of that text (true suffix-array intervals);
 *   "ref"  byte-compatible with the reference builder (genFMindex.c) on any
 *          text: raw-byte suffix order (divbwt64), base2index codes, and for
 *          K >= 2 its LF walk; rows the walk never writes hold code 0 (A)
 *          where the reference leaves uninitialised malloc memory (the
 *          tests emulate its bytes, tests/ref_fill.py).  loadRef also copies the
 *          file the reference's way (readRef, common.c:42-76: later header
 *          lines kept, 255-byte fgets pieces each losing their last byte).
 * All three agree on ACGT-only text. */
int32_t kfmi_set_alphabet(const char *mode);
/* Diagnostics of the last GPU build in this process: sorted positions whose
 * 32-base key tied with their predecessor, and the prefix-doubling rounds the
 * device spent resolving them (0 when there were none). */
int32_t kfmi_build_stats(uint64_t *ties, uint32_t *rounds);

/* Dedup-aware algorithmic traffic of the last search: sum over queries and
 * steps of distinct d-blocks touched (1 if L/d == R/d else 2), SURVEY 8(d). */
int32_t kfmi_count_blocks(void *index, void *queries, uint64_t *blocks);
/* The 128-B lines the active backend's task-kernel fetches touch over the
 * batch (statistics, not timed): out[0] distinct lines per K-step summed over
 * the batch (lines the two ends share counted once), out[1] LF ends whose
 * counter lies outside their planes' line, out[2] LF ends fetched, out[3] ends
 * counted forward from block b-1 (line-local, tags 101/201).  Set the backend
 * and transfer the index first (as for kfmi_count_blocks). */
int32_t kfmi_count_lines(void *index, void *queries, uint64_t out[4]);

/* Streamed search from host memory: `num` queries of `size`
 * ASCII bytes at `ascii`, results [L0,R0,L1,R1,...] into `results` (2*num
 * u32).  The index must already be on the device (transferCPUtoGPU(index,
 * NULL, NULL)).  Chunks of `chunk` queries (0: KFMI_STREAM_CHUNK, else 2^19,
 * or 2^16 when every chunk goes as ASCII) rotate over KFMI_STREAM_SLOTS
 * (default 6) HIP streams so that host packing, H2D, LF and result D2H of
 * successive chunks overlap.  Each
 * chunk either is packed by the host to code words (kfmi_pack_queries; PCIe
 * carries 4 bytes per 16 bases) or goes as ASCII (pinned: DMA'd directly;
 * pageable: staged through pinned buffers) and is packed on the device.  By
 * default the choice is made per chunk from the measured host-packing and
 * link rates (whichever finishes first; KFMI_LINK_SHARERS=n when n processes
 * share the device's PCIe link); KFMI_STREAM_HOSTPACK=1 packs every
 * chunk on the host, =0 sends every chunk as ASCII.  Host work runs on KFMI_HOST_THREADS threads (default min(16,
 * cores)).  Blocking; kfmi_last_timing: total = wall time of the call, pack =
 * host packing / staging time, lf = time blocked on chunks in flight.
 * Results equal kfmi_search's. */
int32_t kfmi_search_stream(void *index, const char *ascii, uint64_t num, uint32_t size,
                           uint32_t *results, uint64_t chunk);
/* loadQueries with the parsing on the device: the file is read
 * in 64 MB pieces into pinned buffers (parallel pread) and DMA'd to the current
 * device, where kernels find the read lines, check them and lay the first
 * `numqueries` reads out as loadQueries would (0 = every read in the file);
 * same format and errors as loadQueries.  The returned queries live on the
 * device only (no host copy): transferCPUtoGPU uses them as they are (on the
 * device they were loaded on); on a device group every member copies its slice
 * device to device, and the parsing device's full copy stays allocated beside
 * the slices (its bytes count twice there) so that the same handle still works
 * in single-device mode afterwards -- freeQueriesGPU releases both. */
int32_t kfmi_load_queries_gpu(const char *fn, uint32_t sizequery, uint64_t numqueries, void **queries);
/* Packs num reads of `size` bases (plain layout q*size, as loadQueries keeps
 * them, common.c:163-173) into the 2-bit code words the search consumes, on the
 * host: word-major, word w of read q at words[w * num + q], ceil(size/16) words
 * per read, the base at reversed index r (base size-1-r) at bits 2r..2r+1 of
 * the read's bit string (fmIndexCPUBaseline.c:200-226 order; K-independent).
 * kfmi_search_stream uses it to send 4 bytes per 16 bases over PCIe. */
int32_t kfmi_pack_queries(const char *ascii, uint64_t num, uint32_t size, uint32_t *words);
/* The same for a K-step index (K = 1, 2 or 4) and reads of any length: with
 * r = size % K, the stream covers bases 0 .. size-r-1 (ceil((size-r)/16) word
 * rows) and, when r > 0, one more row holds each read's remainder-table index
 * (base size-1 at bits 0-1, size-2 at 2-3, ...) -- what kfmi_search_stream
 * sends for such reads.  r = 0 gives kfmi_pack_queries' words. */
int32_t kfmi_pack_queries_k(const char *ascii, uint64_t num, uint32_t size, uint32_t k, uint32_t *words);
/* Host threads of the parallel host paths (loadQueries, the streamed search's
 * packers, the device loader's reads): KFMI_HOST_THREADS, else this process's
 * CPUs (affinity mask capped by the cgroup quota) divided among the ranks on
 * this host (LOCAL_WORLD_SIZE), 2 to 16. */
int32_t kfmi_host_threads(void);
/* Pinned (page-locked) host memory for query/result buffers. */
int32_t kfmi_host_alloc(uint64_t bytes, void **p);
int32_t kfmi_host_free(void *p);
/* Frees the staging and device buffers kfmi_search_stream keeps per device. */
int32_t kfmi_stream_release(void);
/* Share of the reads of this thread's last kfmi_search_stream that were packed
 * on the host (the rest went over PCIe as ASCII). */
double  kfmi_stream_hostpacked_fraction(void);

/* Diagnostic (not in the reference): replays the line requests a
 * task-mid / coop-mid search of `queries` makes (MID128 layout, K = 2, d = 64,
 * m % K == 0, both uploaded) without the LF chain's dependence: a trace launch
 * records every (K-step, read) end's line, then `reps` timed replay launches
 * issue the task kernel's loads for them with `unroll` (1, 2, 4, 8) K-steps in
 * flight per lane, as `groups` (1, 2) exec-masked lane groups (unroll 0: the
 * task kernel's own asm fetch, one K-step in flight).  *ms: mean replay launch time; *lines: lines fetched per
 * launch (= kfmi_count_blocks); *trace_bytes: the trace streamed beside them. */
int32_t kfmi_probe_replay(void *index, void *queries, int32_t unroll, int32_t groups, int32_t reps, double *ms,
                          uint64_t *lines, uint64_t *trace_bytes);

/* Bytes of the device-resident index for the current backend (incl. SA samples). */
uint64_t kfmi_device_index_bytes(void *index);

/* ---- locate: SA interval -> text positions --------------
 * Not in the reference, which stops at [L, R) (fmIndexCPUBaseline.c:288-290).
 * The index keeps a row-sampled suffix array, SA[r] for rows r % rate == 0
 * (rate a power of two <= 65536; 1 = the full SA, 4 B per row), and every other
 * row is walked back with LF_K to a sampled or '$' row on the device. */

/* kfmi_build_index_cpu/_gpu plus SA samples (sa_rate 0: none); `on_device`
 * selects the GPU builder. */
int32_t kfmi_build_index_ex(const char *text, uint64_t n, uint32_t k, uint32_t d, uint32_t sa_rate,
                            int32_t on_device, void **index);
/* The index's samples (count 0 / rate 0 when it has none); owned by the index. */
int32_t kfmi_index_sa(void *index, const uint32_t **sa, uint64_t *count, uint32_t *rate);
/* Sample file: u32 "KSA1", rate, bwtsize, 0; u64 count; u32 samples[count].
 * kfmi_load_sa attaches a file's samples to an index of the same text. */
int32_t kfmi_save_sa(const char *fn, void *index);
int32_t kfmi_load_sa(const char *fn, void *index);
/* Text positions of the rows of every query's [L, R) -- at most max_occ per
 * query (the first rows; 0 = all) -- from results still on the device (after
 * searchIndexGPU / kfmi_search) and an index with samples on the device.
 * Query q's positions are positions[offsets[q] .. offsets[q+1]), in row order
 * (positions[offsets[q] + j] = SA[L_q + j]).  Rows from n+1 on hold no
 * suffix and are not reported (an AltCounters interval can end past n+1).
 * Before the first walk on a device copy, the walk check (kfmi_set_walk_check:
 * one LF_K per row, then the sampled check or pointer jumping; 0.16 s at 3
 * Gbase) verifies that every LF_K walk ends at a '$' row; an index that fails
 * it ('ref'-mode indexes of texts with bytes other than A/C/G/T, whose walks
 * can cycle and would never end) returns KFMI_E_BUILDING_FMI (9) instead of
 * walking, so no slot ever runs the walk_lost cap of n/K steps.  kfmi_last_timing: total, scan, locate kernel (ms).  Errors: 34
 * before transfer/search, 33 without samples, 9 as above. */
int32_t         kfmi_locate(void *index, void *results, uint32_t max_occ, void **locations);
uint64_t        kfmi_locations_total(void *locations);
const uint64_t *kfmi_locations_offsets(void *locations);    /* num + 1 */
const uint32_t *kfmi_locations_positions(void *locations);  /* total */
int32_t         kfmi_locations_free(void **locations);

#ifdef __cplusplus
}
#endif

#endif /* KSTEP_FMI_H_ */
