// cog_abi.cpp -- host side of libcog_hip.so: implements the C ABI of include/cog.h on top of the
// kernels in cog_engine.hip.  No CPU fallback exists: without a gfx950 device every constructor
// fails with COG_ERR_NODEVICE.
//
// A handle owns one or more shards: contiguous env ranges, each resident on one GPU with its own
// HIP stream and device state (the reference ThreadedRunner's contiguous per-worker blocks,
// runner.h:33-38, with GPUs in place of pinned threads).  Seeds are seed + global index, so the
// results do not depend on the shard layout.  Host views are pinned; shard k copies into its
// slice.  Every operation is issued on all shards' streams first and waited for afterwards, so
// the GPUs of a handle run concurrently.
//
// Device layout per shard (one allocation `outs`, padded to 16 B):
//   [status 64 B][selected masks n x 128][infos n x 192][rewards n x 16][dones n][agents n]
// Host views are pinned, device-mapped, coherent memory.  A host-visible call ends with one
// publish kernel per shard (cog_engine.hip k_publish): the ObsData tails and this block are
// compared with an HBM copy of what the host views hold, and the granules that changed are
// stored straight into the views -- no D2H copy commands.  Actions and masks the caller passes
// in the engine's own pinned views are read by the kernels in place (zero-copy); other host
// arrays are staged by an H2D copy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "../../include/cog.h"
#include "cog_engine.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) return fail(COG_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct DeviceGuard {
  int old = -1;
  explicit DeviceGuard(int d) {
    if (hipGetDevice(&old) != hipSuccess) old = -1;
    if (old != d) (void)hipSetDevice(d);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (old >= 0 && hipGetDevice(&cur) == hipSuccess && cur != old) (void)hipSetDevice(old);
  }
};

int check_device(int device) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    return fail(COG_ERR_NODEVICE, "no HIP device available (the engine has no CPU fallback)");
  if (device < 0 || device >= n) return fail(COG_ERR_INVALID, "device ordinal out of range");
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess)
    return fail(COG_ERR_NODEVICE, "hipGetDeviceProperties failed");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(COG_ERR_NODEVICE, std::string("device is ") + prop.gcnArchName +
                                      ", this build targets gfx950 (MI355X) only");
  return COG_OK;
}

template <class T>
int dmalloc(T **p, size_t bytes) {
  if (hipMalloc(reinterpret_cast<void **>(p), bytes ? bytes : 64) != hipSuccess)
    return fail(COG_ERR_OOM, "hipMalloc of " + std::to_string(bytes) + " bytes failed");
  return COG_OK;
}
template <class T>
int hmalloc(T **p, size_t bytes, unsigned flags = hipHostMallocDefault) {
  if (hipHostMalloc(reinterpret_cast<void **>(p), bytes ? bytes : 64, flags) != hipSuccess)
    return fail(COG_ERR_OOM, "hipHostMalloc of " + std::to_string(bytes) + " bytes failed");
  return COG_OK;
}

// Pinned, device-mapped, coherent host memory (uncached on the GPU: kernels read what the host
// last wrote).  Registered so that a caller's pointer into one of these views can be handed to a
// kernel without a staging copy.
constexpr unsigned kZcFlags = hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable;
struct ZcRange {
  const uint8_t *base;
  size_t bytes;
  const uint8_t *dev;                 // the device address of base
  uint64_t same = 0, differs = 0;     // devices (bits) checked to map base at `dev` / elsewhere
};
std::mutex g_zc_mu;
std::vector<ZcRange> g_zc;

template <class T>
int zc_alloc(T **p, size_t bytes) {
  int rc = hmalloc(p, bytes, kZcFlags);
  if (rc) return rc;
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, *p, 0) != hipSuccess) d = nullptr;
  std::lock_guard<std::mutex> lk(g_zc_mu);
  g_zc.push_back({reinterpret_cast<const uint8_t *>(*p), bytes ? bytes : 64, static_cast<const uint8_t *>(d)});
  return COG_OK;
}
void zc_free(void *p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(g_zc_mu);
    for (size_t j = 0; j < g_zc.size(); j++)
      if (g_zc[j].base == p) {
        g_zc.erase(g_zc.begin() + (long)j);
        break;
      }
  }
  (void)hipHostFree(p);
}
// the device address of [p, p + bytes) when the range lies inside one of the engine's mapped
// views, else nullptr (the caller stages a copy)
const uint8_t *zc_device(const void *p, size_t bytes) {
  const uint8_t *q = static_cast<const uint8_t *>(p);
  std::lock_guard<std::mutex> lk(g_zc_mu);
  for (const ZcRange &r : g_zc)
    if (r.dev && q >= r.base && q + bytes <= r.base + r.bytes) return r.dev + (q - r.base);
  return nullptr;
}
// every device of a multi-GPU handle must see a view at the address recorded at allocation;
// the answer is cached per view and device, so the per-step host calls pay one lookup
bool zc_same_on(int device, const void *p) {
  const uint8_t *q = static_cast<const uint8_t *>(p);
  const uint64_t bit = device >= 0 && device < 64 ? 1ull << device : 0;
  const uint8_t *base = nullptr, *expect = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_zc_mu);
    for (const ZcRange &r : g_zc)
      if (r.dev && q >= r.base && q < r.base + r.bytes) {
        if (r.same & bit) return true;
        if (r.differs & bit) return false;
        base = r.base;
        expect = r.dev;
        break;
      }
  }
  if (!base) return false;
  void *d = nullptr;
  bool ok;
  {
    DeviceGuard g(device);
    ok = hipHostGetDevicePointer(&d, const_cast<uint8_t *>(base), 0) == hipSuccess && d == expect;
  }
  std::lock_guard<std::mutex> lk(g_zc_mu);
  for (ZcRange &r : g_zc)   // (the same allocation: a view freed and re-allocated at `base` meanwhile
    if (r.base == base && r.dev == expect) (ok ? r.same : r.differs) |= bit;   // may map elsewhere)
  return ok;
}

// Completion of a host call.  A synchronous call queues k_signal(seq) behind its work and spins
// on the pinned word it stores, instead of hipStreamSynchronize: the word lands about 2.5 us
// before the runtime's own completion signal would wake a stream sync, and a stream sync after
// the spin would wait for that signal again (+8 us measured: profiles/r03_latprobe.txt).  Only
// calls whose results are in device memory or in the engine's pinned views use it (no pageable
// copy is pending).  After spin_us without the word (a long call, or a fault that keeps the
// signal from running), the call falls back to hipStreamSynchronize, which reports errors.
// $COG_SPIN_US sets the spin budget (default 2,000 us; 0: always hipStreamSynchronize).
// A call whose last kernel can store the word itself (k_sample, k_publish: GridSignal, the last
// workgroup through a device counter) arms it instead (signal_arm / signal_armed): one dependent
// dispatch less, about 3 us.
struct Signal {
  volatile uint32_t *h = nullptr;     // host address of the word
  uint32_t *d = nullptr;              // its device address
  uint32_t *ctr = nullptr;            // device counter of the in-kernel form (zero between calls)
  uint32_t seq = 0;
  bool queued = false;                // a store of seq is queued on the stream
};
long spin_budget_us() {
  static const long v = [] {
    const char *e = std::getenv("COG_SPIN_US");
    return e ? std::max(0L, std::atol(e)) : 2000L;
  }();
  return v;
}
// the counter and seq for a kernel that stores the word itself (null: no spinning)
uint32_t *signal_arm(const Signal &g, uint32_t &seq) {
  if (!g.d || !g.ctr || spin_budget_us() <= 0) return nullptr;
  seq = g.seq + 1;
  return g.ctr;
}
void signal_armed(Signal &g) {        // (after the kernel that stores it was launched)
  g.seq++;
  g.queued = true;
}
int signal_enqueue(Signal &g, hipStream_t st) {
  if (g.queued) return COG_OK;                             // (armed in the call's last kernel)
  if (!g.d || spin_budget_us() <= 0) return COG_OK;
  if (cog::launch_signal(g.d, g.seq + 1, st)) {            // (not queued: the wait syncs the stream)
    (void)hipGetLastError();
    return COG_OK;
  }
  g.seq++;
  g.queued = true;
  return COG_OK;
}
// the word, read with acquire semantics: the caller's later plain reads of the pinned views and
// status words are not hoisted above it (x86 orders the loads; this orders the compiler)
bool signal_seen(const Signal &g) {
  return __atomic_load_n(const_cast<const uint32_t *>(g.h), __ATOMIC_ACQUIRE) == g.seq;
}
int signal_wait(Signal &g, hipStream_t st) {
  const bool was_queued = g.queued;
  if (g.queued) {
    g.queued = false;
    if (signal_seen(g)) return COG_OK;
    const auto t0 = std::chrono::steady_clock::now();
    const auto budget = std::chrono::microseconds(spin_budget_us());
    for (unsigned it = 1;; it++) {
      if (signal_seen(g)) return COG_OK;
      __builtin_ia32_pause();
      if (!(it & 255u) && std::chrono::steady_clock::now() - t0 > budget) break;
    }
  }
  HIPCHK(hipStreamSynchronize(st));
  // A kernel that stopped before all its workgroups arrived leaves the in-kernel counter non-zero,
  // and the next armed kernel would store its word early: re-arm the counter whenever a queued
  // word did not land by the time the stream drained.
  if (was_queued && g.ctr && !signal_seen(g)) {
    HIPCHK(hipMemsetAsync(g.ctr, 0, sizeof(uint32_t), st));
    HIPCHK(hipStreamSynchronize(st));
  }
  return COG_OK;
}

// the reference runner's block split (runner.h:33-38): n / k per block, the last takes the rest
std::vector<size_t> block_split(size_t n, int k) {
  std::vector<size_t> first(k + 1);
  const size_t b = n / (size_t)k;
  for (int j = 0; j < k; j++) first[j] = b * (size_t)j;
  first[k] = n;
  return first;
}

constexpr size_t kStatusBytes = 64;
struct OutLayout {                    // offsets inside a shard's `outs` block (device and host)
  size_t sel, info, rew, done, agent, total, alloc;
  explicit OutLayout(size_t n) {
    sel = kStatusBytes;
    info = sel + n * COG_MASK_BYTES;
    rew = info + n * COG_INFO_BYTES;
    done = rew + n * 4 * sizeof(float);
    agent = done + n;
    total = agent + n;
    alloc = (total + 15) & ~(size_t)15;   // whole granules: the publish kernel moves 16 B at a time
  }
};

}  // namespace

struct EnvShard {
  int device = 0;
  size_t first = 0, n = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev = nullptr;            // cross-stream ordering (cog_env_wait_stream / signal_stream)
  cog::DevState s{};
  uint8_t *outs = nullptr;            // device block: status | sel | info | rew | done | agent
  uint8_t *h_outs = nullptr;          // pinned host mirror of `outs`
  uint8_t *d_actions = nullptr;       // staging for host-provided actions
  bool status_dirty = false;          // device status words may be non-zero
  // publish path (host views): the device addresses of this shard's slice of the views, and
  // `mir`, an HBM copy of what they hold (valid once a publish stored every granule)
  bool zc = false;
  uint8_t *h_obs_d = nullptr, *h_outs_d = nullptr, *mir = nullptr;
  bool mir_valid = false;
  // the pinned views (tails and outs block) and the mirror equal HBM: set by every publish, cleared
  // by any device work that no publish followed.  A host step then publishes directly
  // (launch_step_pub), and pub_done tells finish() that the step already did.
  bool host_synced = false, pub_done = false;
  Signal done;                        // completion word: word 32 of the shard's error line
  uint32_t park_seq = 0;              // rollout launches with a fix-up so far (DevState::park_par)
  // Steps since the last reset during which only trio rollouts ran (kNotLean: something else ran,
  // or the shard was never reset with >= 3 players).  After a reset every player is lean (no move,
  // free card / move or removes in progress, narrow decks, nobody has won), the selected-mask loop
  // keeps them so -- no moves, purchases or specials -- and the turn counter grows by at most one
  // per step, so no env of the shard can park before lean_clock + K >= max_steps: a trio launch of
  // K steps then needs no k_env_fixup (cog::launch_rollout's no_fixup; the kernel reports a park
  // anyway as an error, F_PARK_NOFIX).
  uint64_t lean_clock = ~0ull;
  // The last launch that wrote decks was a trio rollout (+ its fix-up), so DevState::cdeck / cwide
  // hold every env's decks and the next trio launch may load them instead of the DeckObs records
  // (DevState::cdeck_ok).  Every other deck-writing call (reset, steps, the other rollouts, a
  // device-record invalidation) clears it.
  bool cdeck_ok = false;
};

struct cog_env {
  size_t n = 0;
  uint8_t n_players = 4;              // the batch's players (reset params; the default ctor's 4)
  uint32_t max_steps = 0;             // the last reset's max_steps (0: unknown)
  uint64_t version = 0;               // changes of the env state (SamplerSpec): from a process-wide
                                      // counter, so no two envs ever share a version value
  std::vector<EnvShard> sh;
  uint32_t *h_err = nullptr;          // pinned, device-mapped: one error word per shard (256 B apart)
  // host views: obs is one pinned allocation; the small records are the shard's h_outs block
  // when there is one shard, and batch-wide arrays gathered from the blocks otherwise
  bool host = false;
  cog_obs_t *h_obs = nullptr;
  cog_action_mask_t *h_sel = nullptr;
  float *h_rew = nullptr;
  uint8_t *h_done = nullptr;
  uint8_t *h_agent = nullptr;
  cog_info_t *h_info = nullptr;
  std::vector<uint32_t> dirty;
};

struct SamplerShard {
  int device = 0;
  size_t first = 0, n = 0;
  hipStream_t stream = nullptr;
  uint32_t *d_rng = nullptr;
  uint8_t *d_actions = nullptr;
  uint8_t *d_masks = nullptr;         // staging for host-provided masks
  Signal done;                        // completion word (cog_sampler::h_sig)
};

// The speculative next sample (single-shard samplers and envs; cog::SampleSpec).  The reference's
// host loop is `sampler.sample(env.selected_action_masks); env.step(sampler.get_actions())`
// (benchmarks.py:47-51): when env.step gets a sampler's own actions view, the step kernel also
// samples that sampler's next actions from the selected masks the step leaves -- with the
// sampler's own state, into spare buffers -- and the sampler's next sample() of the env's own mask
// view takes them: a host copy of the actions and a swap of the state and device-action buffers,
// no launch.  It applies only while nothing has touched the env or the sampler since (version
// counters), no episode ended in the step (its reset is not speculated), and the sampler's device
// actions were never handed out (a swap would break an alias); otherwise sample() runs as always.
struct SamplerSpec {
  uint32_t *d_rng = nullptr;          // spare state buffer (device)
  uint8_t *d_actions = nullptr;       // spare ActionData records (device)
  uint8_t *h = nullptr;               // pinned, device-mapped: n x 8 B actions, then the invalid word
  cog_env *env = nullptr;             // the env whose step speculated, at version env_version
  uint64_t env_version = 0, version = 0;
  bool ok = false;
};

struct cog_sampler {
  size_t n = 0;
  std::vector<SamplerShard> sh;
  cog_action_t *h_actions = nullptr;  // persistent pinned view, all shards
  uint32_t *h_sig = nullptr;          // pinned, device-mapped: one completion word per shard (256 B apart)
  uint64_t version = 0;               // samples so far (every path)
  uint64_t spec_hits = 0;             // of them, the speculative sample taken
  bool exported = false;              // device actions handed out (cog_sampler_device_actions)
  SamplerSpec spec;
};

struct cog_runner {
  cog_env *env = nullptr;
  cog_sampler *smp = nullptr;
  size_t n_threads = 0;
  uint32_t flags = 0;
  bool pending_sample = false;
  bool timing = false;
  std::vector<std::vector<hipEvent_t>> ev;   // per shard: pairs, one per step() launch or rollout() batch
  size_t ev_used = 0;
  uint64_t timed_launches = 0;        // fused launches covered by the recorded pairs
  int chunk = 1;                      // rollout steps per launch (>1: persistent K-step kernel)
};

namespace {

bool single(const cog_env *e) { return e->sh.size() == 1; }

// cog_env::version: every change of any env's state takes the next value of one process-wide
// counter (with per-env counters starting at 0, an env allocated at a freed env's
// address could reach the version a stale speculation recorded)
std::atomic<uint64_t> g_env_versions{0};
void env_changed(cog_env *e) { e->version = g_env_versions.fetch_add(1, std::memory_order_relaxed) + 1; }

// Envs with host views, for cog_sampler_sample: when the masks it gets are one env shard's own
// pinned selected-mask view on the sampler shard's device, and that shard's views equal HBM
// (host_synced: its last publish stored them), the sampler reads the same records in HBM instead
// of over PCIe.  The views are the env's outputs, handed to Python read-only
// (pybind_module.cpp readonly()), so the bytes in HBM are the bytes of the view.  A step may still
// be in flight on the env's stream (an asynchronous runner.step() publishes itself and keeps
// host_synced): the caller then orders the sampler's stream after it (env_stream_in_flight).
std::mutex g_host_envs_mu;
std::vector<cog_env *> g_host_envs;

void host_env_register(cog_env *e, bool on) {
  std::lock_guard<std::mutex> lk(g_host_envs_mu);
  auto it = std::find(g_host_envs.begin(), g_host_envs.end(), e);
  if (on && it == g_host_envs.end()) g_host_envs.push_back(e);
  if (!on && it != g_host_envs.end()) g_host_envs.erase(it);
}

std::vector<cog_sampler *> g_samplers;   // (under g_host_envs_mu)
void sampler_register(cog_sampler *s, bool on) {
  std::lock_guard<std::mutex> lk(g_host_envs_mu);
  auto it = std::find(g_samplers.begin(), g_samplers.end(), s);
  if (on && it == g_samplers.end()) g_samplers.push_back(s);
  if (!on && it != g_samplers.end()) g_samplers.erase(it);
}
// the single-shard sampler whose pinned actions view `actions` is (null: none)
cog_sampler *sampler_of_actions(const cog_action_t *actions, size_t n) {
  std::lock_guard<std::mutex> lk(g_host_envs_mu);
  for (cog_sampler *s : g_samplers)
    if (s->h_actions == actions && s->n == n && s->sh.size() == 1) return s;
  return nullptr;
}
bool env_alive(const cog_env *e) {
  std::lock_guard<std::mutex> lk(g_host_envs_mu);
  return std::find(g_host_envs.begin(), g_host_envs.end(), e) != g_host_envs.end();
}
EnvShard *env_masks_in_hbm(const cog_action_mask_t *masks, size_t n, int device) {
  if (std::getenv("COG_NO_HBM_MASKS")) return nullptr;    // (A/B)
  std::lock_guard<std::mutex> lk(g_host_envs_mu);
  for (cog_env *e : g_host_envs)
    for (EnvShard &k : e->sh)
      if (e->h_sel + k.first == masks && k.n == n && k.device == device && k.host_synced) return &k;
  return nullptr;
}
// work of the env shard that may still be running on its stream: a step that publishes itself and
// whose completion no sync has consumed yet (pub_done), or any queued completion word
bool env_stream_in_flight(const EnvShard &k) { return k.pub_done || k.done.queued; }

void env_free(cog_env *e) {
  if (!e) return;
  host_env_register(e, false);
  {                                                        // a speculation on this env is void: a new
    std::lock_guard<std::mutex> lk(g_host_envs_mu);        // env at the same address must not match it
    for (cog_sampler *q : g_samplers)
      if (q->spec.env == e) {
        q->spec.ok = false;
        q->spec.env = nullptr;
      }
  }
  for (EnvShard &k : e->sh) {
    DeviceGuard g(k.device);
    if (k.stream) (void)hipStreamSynchronize(k.stream);
    void *dev[] = {k.s.obs, k.outs, k.s.priv, k.s.grid, k.s.cgrid, k.s.heads, k.s.cdeck, k.s.cwide, k.s.gen, k.s.dirty, k.d_actions, k.mir,
                   k.s.park, k.s.parkq, k.done.ctr};
    for (void *p : dev)
      if (p) (void)hipFree(p);
    zc_free(k.h_outs);
    if (k.ev) (void)hipEventDestroy(k.ev);
    if (k.stream) (void)hipStreamDestroy(k.stream);
  }
  zc_free(e->h_obs);
  if (e->h_err) (void)hipHostFree(e->h_err);
  if (!single(e)) {
    void *more[] = {e->h_sel, e->h_rew, e->h_done, e->h_agent, e->h_info};
    for (void *p : more) zc_free(p);
  }
  delete e;
}

int sync_all(cog_env *e) {
  for (EnvShard &k : e->sh) {
    DeviceGuard g(k.device);
    HIPCHK(hipStreamSynchronize(k.stream));
  }
  return COG_OK;
}

// sync_all through the completion words: for calls whose results are in device memory or in
// pinned views (no pageable copy pending)
int sync_fast(cog_env *e) {
  for (EnvShard &k : e->sh) {
    DeviceGuard g(k.device);
    int rc = signal_enqueue(k.done, k.stream);
    if (rc) return rc;
  }
  for (EnvShard &k : e->sh) {
    DeviceGuard g(k.device);
    int rc = signal_wait(k.done, k.stream);
    if (rc) return rc;
  }
  return COG_OK;
}

int status_to_rc(uint32_t flags, uint32_t errors) {
  if (errors) {
    if (flags & cog::F_SYNC_TIMEOUT)
      return fail(COG_ERR_HIP, "internal error: a rollout wave's progress wait timed out (outputs invalid)");
    if (flags & cog::F_PARK_NOFIX)
      return fail(COG_ERR_HIP, "internal error: an env parked in a rollout launched without its fix-up (outputs invalid)");
    if (flags & cog::F_GRID_OVER)
      return fail(COG_ERR_MAPGEN, "map generation produced a map larger than the 48x48 observation grid");
    return fail(COG_ERR_MAPGEN, "Failed to generate map in specified maximum number of attempts");
  }
  return COG_OK;
}

// the D2H copies a host-visible step needs: the ObsData tail (dynamic part: phase, resources,
// shop, decks, stored masks) and the outs block (status words included)
int enqueue_refresh(cog_env *e, EnvShard &k) {
  if (!k.n) return COG_OK;
  HIPCHK(hipMemcpy2DAsync(reinterpret_cast<uint8_t *>(e->h_obs + k.first) + COG_OBS_MAP_BYTES, COG_OBS_BYTES,
                          k.s.obs + COG_OBS_MAP_BYTES, COG_OBS_BYTES, COG_OBS_BYTES - COG_OBS_MAP_BYTES, k.n,
                          hipMemcpyDeviceToHost, k.stream));
  HIPCHK(hipMemcpyAsync(k.h_outs, k.outs, OutLayout(k.n).total, hipMemcpyDeviceToHost, k.stream));
  return COG_OK;
}

int enqueue_status_only(EnvShard &k) {
  HIPCHK(hipMemcpyAsync(k.h_outs, k.outs, kStatusBytes, hipMemcpyDeviceToHost, k.stream));
  return COG_OK;
}

// multi-shard handles keep batch-wide host arrays for the small records: gather the slices
void gather_small(cog_env *e) {
  if (single(e)) return;
  for (EnvShard &k : e->sh) {
    const OutLayout L(k.n);
    std::memcpy(e->h_sel + k.first, k.h_outs + L.sel, k.n * COG_MASK_BYTES);
    std::memcpy(e->h_info + k.first, k.h_outs + L.info, k.n * COG_INFO_BYTES);
    std::memcpy(e->h_rew + 4 * k.first, k.h_outs + L.rew, k.n * 4 * sizeof(float));
    std::memcpy(e->h_done + k.first, k.h_outs + L.done, k.n);
    std::memcpy(e->h_agent + k.first, k.h_outs + L.agent, k.n);
  }
}

// Status after a batch of work.  Device-only work (host views not refreshed) learns "no error"
// from the host-mapped error words after the stream sync, with no copy; host-visible work reads
// the status words that came with its refresh copy.  Regenerated maps (auto-resets) are copied
// to the host views afterwards.  Status words are cleared only when they are non-zero.
int enqueue_publish(EnvShard &k, const SamplerShard *q, uint8_t *h_act_d) {
  if (!k.n) return COG_OK;
  const OutLayout L(k.n);
  uint32_t seq = 0;
  uint32_t *ctr = cog::publish_can_signal(k.n, L.alloc, q && h_act_d) ? signal_arm(k.done, seq) : nullptr;
  if (cog::launch_publish(k.s, k.outs, k.mir, k.h_obs_d, k.h_outs_d, L.alloc, k.mir_valid ? 0 : 1,
                          q ? q->d_actions : nullptr, q ? h_act_d : nullptr, k.stream, ctr, k.done.d, seq))
    return fail(COG_ERR_HIP, std::string("publish launch failed: ") + hipGetErrorString(hipGetLastError()));
  if (ctr) signal_armed(k.done);
  k.mir_valid = true;
  return COG_OK;
}

// smp (optional): a runner's sampler whose actions' host view is refreshed with the env's
int finish(cog_env *e, bool refresh_host, cog_sampler *smp = nullptr) {
  const bool host = refresh_host && e->host;
  for (EnvShard &k : e->sh) {
    if (!k.pub_done) k.done.queued = false;               // (a failed call may have left one armed)
    k.host_synced = false;                                 // (until this call has published)
  }
  for (size_t j = 0; j < e->sh.size(); j++) {
    EnvShard &k = e->sh[j];
    DeviceGuard g(k.device);
    int rc = COG_OK;
    if (k.pub_done) {                                      // the step published itself
      k.pub_done = false;
      continue;
    }
    if (host && k.zc) {
      const SamplerShard *q = smp ? &smp->sh[j] : nullptr;
      uint8_t *h_act = q ? const_cast<uint8_t *>(zc_device(smp->h_actions + q->first, q->n * COG_ACTION_BYTES)) : nullptr;
      if (h_act && !zc_same_on(k.device, smp->h_actions + q->first)) h_act = nullptr;   // this GPU's mapping differs
      if (q && q->n && !h_act)
        HIPCHK(hipMemcpyAsync(smp->h_actions + q->first, q->d_actions, q->n * COG_ACTION_BYTES, hipMemcpyDeviceToHost,
                              k.stream));
      rc = enqueue_publish(k, h_act ? q : nullptr, h_act);
    } else if (host) {
      if (smp && smp->sh[j].n)
        HIPCHK(hipMemcpyAsync(smp->h_actions + smp->sh[j].first, smp->sh[j].d_actions,
                              smp->sh[j].n * COG_ACTION_BYTES, hipMemcpyDeviceToHost, k.stream));
      rc = enqueue_refresh(e, k);
    }
    if (rc) return rc;
  }
  int rc = sync_fast(e);
  if (rc) return rc;
  uint32_t flags = 0, errors = 0;
  bool any_dirty = false;
  for (size_t j = 0; j < e->sh.size(); j++) {
    EnvShard &k = e->sh[j];
    DeviceGuard g(k.device);
    const bool err = e->h_err[64 * j] != 0u;
    if (!host) {
      if (!err) {
        k.status_dirty = true;        // the dirty-map counter may have moved: clear before host use
        continue;
      }
      if ((rc = enqueue_status_only(k))) return rc;
      HIPCHK(hipStreamSynchronize(k.stream));
    }
    const uint32_t *st = reinterpret_cast<const uint32_t *>(k.h_outs);
    const uint32_t st0 = st[0], st1 = st[1], st2 = st[2];
    flags |= st0;
    errors += st1;
    if (host && st2) {
      any_dirty = true;
      if (st2 >= k.n / 8 || st2 > k.s.cap) {   // many resets (or list overflow): copy every map
        HIPCHK(hipMemcpy2DAsync(e->h_obs + k.first, COG_OBS_BYTES, k.s.obs, COG_OBS_BYTES, COG_OBS_MAP_BYTES, k.n,
                                hipMemcpyDeviceToHost, k.stream));
      } else {
        e->dirty.resize(st2);
        HIPCHK(hipMemcpyAsync(e->dirty.data(), k.s.dirty, st2 * sizeof(uint32_t), hipMemcpyDeviceToHost, k.stream));
        HIPCHK(hipStreamSynchronize(k.stream));
        for (uint32_t q = 0; q < st2; q++) {
          const size_t i = e->dirty[q];
          HIPCHK(hipMemcpyAsync(reinterpret_cast<uint8_t *>(e->h_obs + k.first + i), k.s.obs + i * COG_OBS_BYTES,
                                COG_OBS_MAP_BYTES, hipMemcpyDeviceToHost, k.stream));
        }
      }
    }
    if (st0 || st1 || st2 || k.status_dirty || err) {
      HIPCHK(hipMemsetAsync(k.outs, 0, kStatusBytes, k.stream));
      e->h_err[64 * j] = 0u;
      k.status_dirty = false;
    }
  }
  if (any_dirty && (rc = sync_all(e))) return rc;
  if (host) gather_small(e);
  for (EnvShard &k : e->sh) k.host_synced = host && k.zc && k.mir_valid;
  return status_to_rc(flags, errors);
}

// before a host-visible batch: status words still counting from device-only work are cleared
int prepare_host(cog_env *e) {
  for (EnvShard &k : e->sh) {
    if (!k.status_dirty) continue;
    DeviceGuard g(k.device);
    HIPCHK(hipMemsetAsync(k.outs, 0, kStatusBytes, k.stream));
    k.status_dirty = false;
  }
  return COG_OK;
}

int refresh_full(cog_env *e) {
  if (!e->host || !e->n) return COG_OK;
  for (EnvShard &k : e->sh) {
    if (!k.n) continue;
    DeviceGuard g(k.device);
    HIPCHK(hipMemcpyAsync(e->h_obs + k.first, k.s.obs, k.n * COG_OBS_BYTES, hipMemcpyDeviceToHost, k.stream));
    HIPCHK(hipMemcpyAsync(k.h_outs + kStatusBytes, k.outs + kStatusBytes, OutLayout(k.n).total - kStatusBytes,
                          hipMemcpyDeviceToHost, k.stream));
  }
  int rc = sync_all(e);
  if (rc) return rc;
  for (EnvShard &k : e->sh) k.mir_valid = false;   // the views now hold what no mirror recorded
  gather_small(e);
  return COG_OK;
}

// the shard's state as the kernels see it: no dirty-map list unless the host views follow
cog::DevState launch_state(const EnvShard &k, bool host_views) {
  cog::DevState s = k.s;
  if (!host_views) s.cap = 0;
  s.cdeck_ok = k.cdeck_ok ? 1u : 0u;
  return s;
}

void sampler_free(cog_sampler *s) {
  if (!s) return;
  sampler_register(s, false);
  if (!s->sh.empty()) {
    DeviceGuard g(s->sh[0].device);
    if (s->spec.d_rng) (void)hipFree(s->spec.d_rng);
    if (s->spec.d_actions) (void)hipFree(s->spec.d_actions);
  }
  zc_free(s->spec.h);
  for (SamplerShard &k : s->sh) {
    DeviceGuard g(k.device);
    if (k.stream) (void)hipStreamSynchronize(k.stream);
    void *dev[] = {k.d_rng, k.d_actions, k.d_masks, k.done.ctr};
    for (void *p : dev)
      if (p) (void)hipFree(p);
    if (k.stream) (void)hipStreamDestroy(k.stream);
  }
  zc_free(s->h_actions);
  if (s->h_sig) (void)hipHostFree(s->h_sig);
  delete s;
}

int check_devices(const int *devices, int n_devices) {
  if (!devices || n_devices < 1) return fail(COG_ERR_INVALID, "need at least one device");
  for (int j = 0; j < n_devices; j++) {
    int rc = check_device(devices[j]);
    if (rc) return rc;
  }
  return COG_OK;
}

int env_shard_init(EnvShard &k, uint32_t default_seed, uint32_t *err_word) {
  DeviceGuard g(k.device);
  HIPCHK(hipStreamCreateWithFlags(&k.stream, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&k.ev, hipEventDisableTiming));
  const size_t n = k.n;
  const OutLayout L(n);
  cog::DevState &s = k.s;
  int rc;
  if ((rc = dmalloc(&s.obs, n * COG_OBS_BYTES)) || (rc = dmalloc(&k.outs, L.alloc)) ||
      (rc = dmalloc(&s.priv, n * sizeof(cog::EnvPriv))) || (rc = dmalloc(&s.grid, n * (size_t)cog::kGridBytes)) ||
      (rc = dmalloc(&s.cgrid, n * (size_t)COG_CELLS)) || (rc = dmalloc(&s.heads, n * 5 * sizeof(uint4))) ||
      (rc = dmalloc(&s.gen, n * sizeof(cog::GenScratch))) || (rc = dmalloc(&s.dirty, n * sizeof(uint32_t))) ||
      (rc = dmalloc(&k.d_actions, n * COG_ACTION_BYTES)) || (rc = dmalloc(&s.park, n * sizeof(uint32_t))) ||
      (rc = dmalloc(&s.parkq, cog::park_list_bytes(n))) ||
      (rc = dmalloc(&k.done.ctr, 256)) || (rc = zc_alloc(&k.h_outs, L.alloc)) ||
      (rc = dmalloc(&s.cdeck, n * 10 * sizeof(uint4))) || (rc = dmalloc(&s.cwide, n * sizeof(uint32_t))))
    return rc;
  std::memset(k.h_outs, 0, L.alloc);
  s.n = n;
  s.first = k.first;
  s.cap = n;
  s.autoreset = 1;
  s.status = reinterpret_cast<uint32_t *>(k.outs);
  s.sel = k.outs + L.sel;
  s.info = k.outs + L.info;
  s.rew = reinterpret_cast<float *>(k.outs + L.rew);
  s.done = k.outs + L.done;
  s.agent = k.outs + L.agent;
  void *d_err = nullptr;
  HIPCHK(hipHostGetDevicePointer(&d_err, err_word, 0));
  s.err = static_cast<uint32_t *>(d_err);
  k.done.h = err_word + 32;
  k.done.d = s.err + 32;
  struct { void *p; size_t b; } z[] = {{s.obs, n * COG_OBS_BYTES}, {k.outs, L.alloc}, {s.grid, n * (size_t)cog::kGridBytes},
                                       {s.cgrid, n * (size_t)COG_CELLS}, {s.gen, n * sizeof(cog::GenScratch)},
                                       {k.d_actions, n * COG_ACTION_BYTES}, {k.done.ctr, 256}};
  for (auto &zz : z)
    if (zz.b) HIPCHK(hipMemsetAsync(zz.p, 0, zz.b, k.stream));
  if (n) HIPCHK(hipMemsetAsync(s.park, 0xff, n * sizeof(uint32_t), k.stream));   // no env parked
  HIPCHK(hipMemsetAsync(s.parkq, 0, cog::park_list_bytes(n), k.stream));          // both counters 0
  if (cog::launch_init(s, nullptr, default_seed, k.stream))
    return fail(COG_ERR_HIP, std::string("env init kernel failed: ") + hipGetErrorString(hipGetLastError()));
  return COG_OK;
}

int shard_of(const cog_env *e, int k) {
  if (!e || k < 0 || (size_t)k >= e->sh.size()) return fail(COG_ERR_INVALID, "shard index out of range");
  return COG_OK;
}

}  // namespace

extern "C" {

const char *cog_last_error(void) { return g_err.c_str(); }
int cog_abi_version(void) { return COG_ABI_VERSION; }
int cog_rollout_kind(size_t n_envs, int n_players, int stored_masks) {
  return cog::rollout_kind_of(n_envs, stored_masks ? cog::MASK_STORED : cog::MASK_SELECTED, n_players >= 3);
}

int cog_device_count(int *out) {
  if (!out) return fail(COG_ERR_INVALID, "out is NULL");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *out = n;
  return COG_OK;
}

int cog_env_create_multi(size_t n_envs, const int *devices, int n_devices, cog_env **out) {
  if (!out) return fail(COG_ERR_INVALID, "out is NULL");
  *out = nullptr;
  int rc = check_devices(devices, n_devices);
  if (rc) return rc;
  cog_env *e = new cog_env();
  e->n = n_envs;
  env_changed(e);
  const size_t err_bytes = 64 * sizeof(uint32_t) * (size_t)n_devices;
  if ((rc = hmalloc(&e->h_err, err_bytes, hipHostMallocMapped | hipHostMallocCoherent))) {
    env_free(e);
    return rc;
  }
  std::memset(e->h_err, 0, err_bytes);
  const std::vector<size_t> first = block_split(n_envs, n_devices);
  const uint32_t default_seed = std::random_device{}();   // cog_env() seeds from random_device
  e->sh.resize(n_devices);
  for (int j = 0; j < n_devices; j++) {
    EnvShard &k = e->sh[j];
    k.device = devices[j];
    k.first = first[j];
    k.n = first[j + 1] - first[j];
    if ((rc = env_shard_init(k, default_seed, e->h_err + 64 * j))) {   // one 256-B line per shard
      env_free(e);
      return rc;
    }
  }
  if ((rc = sync_all(e))) {
    env_free(e);
    return rc;
  }
  *out = e;
  return COG_OK;
}

int cog_env_create(size_t n_envs, int device, cog_env **out) { return cog_env_create_multi(n_envs, &device, 1, out); }

void cog_env_destroy(cog_env *env) { env_free(env); }

int cog_env_num_envs(const cog_env *env, size_t *out) {
  if (!env || !out) return fail(COG_ERR_INVALID, "NULL argument");
  *out = env->n;
  return COG_OK;
}

int cog_env_num_shards(const cog_env *env, int *out) {
  if (!env || !out) return fail(COG_ERR_INVALID, "NULL argument");
  *out = (int)env->sh.size();
  return COG_OK;
}

int cog_env_shard_info(const cog_env *env, int k, size_t *first, size_t *count, int *device) {
  int rc = shard_of(env, k);
  if (rc) return rc;
  const EnvShard &s = env->sh[k];
  if (first) *first = s.first;
  if (count) *count = s.n;
  if (device) *device = s.device;
  return COG_OK;
}

static int env_reset_impl(cog_env *e, const cog::ResetParams &p) {
  int rc = prepare_host(e);
  if (rc) return rc;
  env_changed(e);
  if (p.use_params) {
    e->n_players = p.n_players;
    e->max_steps = p.max_steps;
  }
  for (EnvShard &k : e->sh) {
    k.done.queued = false;
    k.host_synced = false;                                 // (refresh_full: the mirror is rebuilt later)
    k.lean_clock = e->n_players >= 3 && e->max_steps ? 0ull : ~0ull;
    k.cdeck_ok = false;
  }
  for (EnvShard &k : e->sh) {
    DeviceGuard g(k.device);
    if (cog::launch_reset(k.s, p, k.stream) || cog::launch_encode_all(k.s, k.stream))
      return fail(COG_ERR_HIP, std::string("reset launch failed: ") + hipGetErrorString(hipGetLastError()));
    if ((rc = enqueue_status_only(k))) return rc;
  }
  if ((rc = sync_fast(e))) return rc;
  uint32_t flags = 0, errors = 0;
  for (size_t j = 0; j < e->sh.size(); j++) {
    EnvShard &k = e->sh[j];
    const uint32_t *st = reinterpret_cast<const uint32_t *>(k.h_outs);
    flags |= st[0];
    errors += st[1];
    if (st[0] || st[1] || st[2] || e->h_err[64 * j]) {
      DeviceGuard g(k.device);
      HIPCHK(hipMemsetAsync(k.outs, 0, kStatusBytes, k.stream));
      e->h_err[64 * j] = 0u;
    }
  }
  if ((rc = refresh_full(e))) return rc;
  return status_to_rc(flags, errors);
}

int cog_env_reset(cog_env *env, uint32_t seed, uint8_t n_players, uint8_t n_pieces, int32_t difficulty,
                  uint32_t max_steps, int32_t render) {
  if (!env) return fail(COG_ERR_INVALID, "env is NULL");
  if (n_players < 1 || n_players > COG_MAX_N_PLAYERS_)
    return fail(COG_ERR_INVALID, "n_players must be in 1..4");
  if (difficulty < COG_EASY || difficulty > COG_HARD) return fail(COG_ERR_INVALID, "invalid difficulty");
  (void)render;
  cog::ResetParams p{seed, n_players, n_pieces, (uint8_t)difficulty, 1, max_steps};
  return env_reset_impl(env, p);
}

int cog_env_reset_default(cog_env *env) {
  if (!env) return fail(COG_ERR_INVALID, "env is NULL");
  cog::ResetParams p{0, 0, 0, 0, 0, 0};
  return env_reset_impl(env, p);
}

int cog_env_step_device_stream(cog_env *env, const void *d_actions, size_t n, void *stream) {
  if (!env || !d_actions) return fail(COG_ERR_INVALID, "NULL argument");
  if (n != env->n) return fail(COG_ERR_INVALID, "actions length != num_envs");
  if (!single(env)) return fail(COG_ERR_INVALID, "device actions need a single-shard env (one device pointer)");
  EnvShard &k = env->sh[0];
  DeviceGuard g(k.device);
  int rc = prepare_host(env);
  if (rc) return rc;
  env_changed(env);
  if (stream != COG_NO_STREAM) {      // the caller's stream produced the actions: order after it
    HIPCHK(hipEventRecord(k.ev, static_cast<hipStream_t>(stream)));   // (NULL: the null stream)
    HIPCHK(hipStreamWaitEvent(k.stream, k.ev, 0));
  }
  k.lean_clock = ~0ull;                                    // (arbitrary actions)
  k.cdeck_ok = false;
  if (cog::launch_step(launch_state(k, env->host), static_cast<const uint8_t *>(d_actions), k.stream))
    return fail(COG_ERR_HIP, std::string("step launch failed: ") + hipGetErrorString(hipGetLastError()));
  return finish(env, true);
}

int cog_env_step_device(cog_env *env, const void *d_actions, size_t n) {
  return cog_env_step_device_stream(env, d_actions, n, COG_NO_STREAM);
}

// spare buffers of a single-shard sampler for the speculative sample (allocated on first use)
static bool spec_ready(cog_sampler *q) {
  SamplerSpec &sp = q->spec;
  if (sp.h) return true;
  DeviceGuard g(q->sh[0].device);
  if (dmalloc(&sp.d_rng, q->n * sizeof(uint32_t)) || dmalloc(&sp.d_actions, q->n * COG_ACTION_BYTES) ||
      zc_alloc(&sp.h, q->n * 8 + 64)) {
    (void)hipGetLastError();
    return false;
  }
  std::memset(sp.h, 0, q->n * 8 + 64);
  return hipMemset(sp.d_actions, 0, q->n * COG_ACTION_BYTES) == hipSuccess;
}

int cog_env_step(cog_env *env, const cog_action_t *actions, size_t n) {
  if (!env || (!actions && n)) return fail(COG_ERR_INVALID, "NULL argument");
  if (n != env->n) return fail(COG_ERR_INVALID, "actions length != num_envs");
  int rc = prepare_host(env);
  if (rc) return rc;
  env_changed(env);
  // the actions are a sampler's own view: its next sample, speculatively (SamplerSpec)
  cog_sampler *q = single(env) && n ? sampler_of_actions(actions, n) : nullptr;
  if (q && (q->exported || q->sh[0].device != env->sh[0].device || std::getenv("COG_NO_SPEC") || !spec_ready(q)))
    q = nullptr;
  if (q) q->spec.ok = false;
  bool spec_launched = false;
  for (EnvShard &k : env->sh) {
    if (!k.n) continue;
    DeviceGuard g(k.device);
    const uint8_t *da = zc_device(actions + k.first, k.n * COG_ACTION_BYTES);   // read in place when pinned
    if (!da || !zc_same_on(k.device, actions + k.first)) {                      // (and mapped alike on this GPU)
      HIPCHK(hipMemcpyAsync(k.d_actions, actions + k.first, k.n * COG_ACTION_BYTES, hipMemcpyHostToDevice, k.stream));
      da = k.d_actions;
    }
    uint32_t seq = 0, *ctr = nullptr;
    k.pub_done = false;
    k.lean_clock = ~0ull;                                  // (arbitrary actions)
    k.cdeck_ok = false;
    if (env->host && k.zc && k.mir_valid && k.host_synced && cog::step_pub_ok(k.n) &&
        (ctr = signal_arm(k.done, seq))) {                 // the step publishes and signals itself
      cog::DevState ps = launch_state(k, true);
      ps.pub_obs = k.h_obs_d;
      ps.pub_outs = k.h_outs_d;
      ps.pub_mir = k.mir;
      cog::SampleSpec sp{nullptr, nullptr, nullptr, nullptr, nullptr};
      if (q) {
        uint8_t *h = const_cast<uint8_t *>(zc_device(q->spec.h, n * 8 + 64));
        if (h) {
          *reinterpret_cast<volatile uint32_t *>(q->spec.h + n * 8) = 0u;   // the invalid word
          sp = cog::SampleSpec{q->sh[0].d_rng, q->spec.d_rng, q->spec.d_actions, h, reinterpret_cast<uint32_t *>(h + n * 8)};
          spec_launched = true;
        }
      }
      if (cog::launch_step_pub(ps, da, k.stream, ctr, k.done.d, seq, spec_launched ? &sp : nullptr))
        return fail(COG_ERR_HIP, std::string("step launch failed: ") + hipGetErrorString(hipGetLastError()));
      signal_armed(k.done);
      k.pub_done = true;
      continue;
    }
    if (cog::launch_step(launch_state(k, env->host), da, k.stream))
      return fail(COG_ERR_HIP, std::string("step launch failed: ") + hipGetErrorString(hipGetLastError()));
  }
  rc = finish(env, true);
  if (!rc && spec_launched) {                              // the step has completed: its speculation stands
    q->spec.env = env;
    q->spec.env_version = env->version;
    q->spec.version = q->version;
    q->spec.ok = true;
  }
  return rc;
}

static int alloc_host_views(cog_env *env) {
  const size_t n = env->n;
  int rc;
  if ((rc = zc_alloc(&env->h_obs, n * COG_OBS_BYTES))) return rc;
  std::memset(env->h_obs, 0, n * COG_OBS_BYTES);   // padding bytes stay defined
  if (single(env)) {                                // views point straight into the copy target
    EnvShard &k = env->sh[0];
    const OutLayout L(k.n);
    env->h_sel = reinterpret_cast<cog_action_mask_t *>(k.h_outs + L.sel);
    env->h_info = reinterpret_cast<cog_info_t *>(k.h_outs + L.info);
    env->h_rew = reinterpret_cast<float *>(k.h_outs + L.rew);
    env->h_done = k.h_outs + L.done;
    env->h_agent = k.h_outs + L.agent;
  } else if ((rc = zc_alloc(&env->h_sel, n * COG_MASK_BYTES)) || (rc = zc_alloc(&env->h_rew, n * 4 * sizeof(float))) ||
             (rc = zc_alloc(&env->h_done, n)) || (rc = zc_alloc(&env->h_agent, n)) ||
             (rc = zc_alloc(&env->h_info, n * COG_INFO_BYTES))) {
    return rc;
  }
  for (EnvShard &k : env->sh) {                     // the publish path, where every device maps the views
    if (!k.n) continue;
    const OutLayout L(k.n);
    k.h_obs_d = const_cast<uint8_t *>(zc_device(env->h_obs + k.first, k.n * COG_OBS_BYTES));
    k.h_outs_d = const_cast<uint8_t *>(zc_device(k.h_outs, L.alloc));
    DeviceGuard g(k.device);
    k.zc = k.h_obs_d && k.h_outs_d && zc_same_on(k.device, env->h_obs) && zc_same_on(k.device, k.h_outs) &&
           !std::getenv("COG_NO_ZEROCOPY");
    if (k.zc && (rc = dmalloc(&k.mir, cog::publish_mirror_bytes(k.n, L.alloc)))) return rc;
    k.mir_valid = false;
  }
  env->host = true;
  host_env_register(env, true);
  return refresh_full(env);
}

int cog_env_get_views(cog_env *env, cog_env_views *out) {
  if (!env || !out) return fail(COG_ERR_INVALID, "NULL argument");
  if (!env->host) {
    int rc = alloc_host_views(env);
    if (rc) return rc;
  }
  std::memset(out, 0, sizeof(*out));
  out->n_envs = env->n;
  out->observations = env->h_obs;
  out->selected_action_masks = env->h_sel;
  out->rewards = env->h_rew;
  out->dones = env->h_done;
  out->agent_selection = env->h_agent;
  out->infos = env->h_info;
  if (single(env)) {                                // device views: one device pointer per record kind
    const EnvShard &k = env->sh[0];
    out->d_observations = k.s.obs;
    out->d_selected_action_masks = k.s.sel;
    out->d_rewards = k.s.rew;
    out->d_dones = k.s.done;
    out->d_agent_selection = k.s.agent;
    out->d_infos = k.s.info;
  }
  return COG_OK;
}

int cog_env_shard_views(cog_env *env, int k, cog_env_views *out) {
  int rc = shard_of(env, k);
  if (rc) return rc;
  if (!out) return fail(COG_ERR_INVALID, "NULL argument");
  cog_env_views all;
  if ((rc = cog_env_get_views(env, &all))) return rc;
  const EnvShard &s = env->sh[k];
  std::memset(out, 0, sizeof(*out));
  out->n_envs = s.n;
  out->observations = all.observations + s.first;
  out->selected_action_masks = all.selected_action_masks + s.first;
  out->rewards = all.rewards + 4 * s.first;
  out->dones = all.dones + s.first;
  out->agent_selection = all.agent_selection + s.first;
  out->infos = all.infos + s.first;
  out->d_observations = s.s.obs;
  out->d_selected_action_masks = s.s.sel;
  out->d_rewards = s.s.rew;
  out->d_dones = s.s.done;
  out->d_agent_selection = s.s.agent;
  out->d_infos = s.s.info;
  return COG_OK;
}

int cog_env_sync_host(cog_env *env) {
  if (!env) return fail(COG_ERR_INVALID, "env is NULL");
  if (!env->host) return alloc_host_views(env);
  return refresh_full(env);
}

int cog_env_hazards(cog_env *env, uint32_t *flags_or, uint32_t *per_env) {
  if (!env) return fail(COG_ERR_INVALID, "env is NULL");
  std::vector<uint32_t> tmp(env->n);
  for (EnvShard &k : env->sh) {
    if (!k.n) continue;
    DeviceGuard g(k.device);
    HIPCHK(hipMemcpy2DAsync(tmp.data() + k.first, sizeof(uint32_t),
                            reinterpret_cast<uint8_t *>(k.s.priv) + offsetof(cog::EnvPriv, flags), sizeof(cog::EnvPriv),
                            sizeof(uint32_t), k.n, hipMemcpyDeviceToHost, k.stream));
  }
  int rc = sync_all(env);
  if (rc) return rc;
  uint32_t acc = 0;
  for (uint32_t f : tmp) acc |= f;
  if (flags_or) *flags_or = acc;
  if (per_env) std::memcpy(per_env, tmp.data(), tmp.size() * sizeof(uint32_t));
  return COG_OK;
}

int cog_env_clear_hazards(cog_env *env) {
  if (!env) return fail(COG_ERR_INVALID, "env is NULL");
  for (EnvShard &k : env->sh) {
    if (!k.n) continue;
    DeviceGuard g(k.device);
    HIPCHK(hipMemset2DAsync(reinterpret_cast<uint8_t *>(k.s.priv) + offsetof(cog::EnvPriv, flags), sizeof(cog::EnvPriv),
                            0, sizeof(uint32_t), k.n, k.stream));
  }
  return sync_all(env);
}

int cog_env_time_encode(cog_env *env, int iters, int variant, double *ms_per_launch) {
  if (!env || iters < 1 || !ms_per_launch) return fail(COG_ERR_INVALID, "bad argument");
  EnvShard &k = env->sh[0];                         // diagnostic: shard 0
  DeviceGuard g(k.device);
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  if (cog::launch_encode_all(k.s, k.stream, variant))   // warm-up launch
    return fail(COG_ERR_HIP, "encode launch failed");
  HIPCHK(hipEventRecord(e0, k.stream));
  for (int r = 0; r < iters; r++)
    if (cog::launch_encode_all(k.s, k.stream, variant)) return fail(COG_ERR_HIP, "encode launch failed");
  HIPCHK(hipEventRecord(e1, k.stream));
  HIPCHK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  *ms_per_launch = (double)ms / iters;
  return COG_OK;
}

static int time_copy_variants(int device, size_t bytes, int iters, double *gb_per_s, bool mix);
int cog_time_copy(int device, size_t bytes, int iters, double *gb_per_s) {
  return time_copy_variants(device, bytes, iters, gb_per_s, false);
}
int cog_time_stream_mix(int device, size_t bytes, int iters, double *gb_per_s) {
  return time_copy_variants(device, bytes, iters, gb_per_s, true);
}
static int time_copy_variants(int device, size_t bytes, int iters, double *gb_per_s, bool mix) {
  if (iters < 1 || bytes < 16 || !gb_per_s) return fail(COG_ERR_INVALID, "bad argument");
  bytes &= ~(size_t)15;
  int cnt = 0;
  if (hipGetDeviceCount(&cnt) != hipSuccess || device < 0 || device >= cnt) return fail(COG_ERR_NODEVICE, "no HIP device");
  DeviceGuard g(device);
  void *a = nullptr, *b = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = COG_OK;
  const size_t out_bytes = mix ? 7 * bytes : bytes;      // (mix: `bytes` read, 7x written)
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, out_bytes) != hipSuccess) rc = fail(COG_ERR_OOM, "copy buffers");
  if (!rc && (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
              hipEventCreate(&e1) != hipSuccess || hipMemsetAsync(a, 1, bytes, st) != hipSuccess))
    rc = fail(COG_ERR_HIP, "copy setup");
  double best = 0.0;
  // the fastest variant: copy 0-7 (grid stride / one pass, plain / non-temporal) and 16-17 (one
  // granule per work-item); the mix 8-9
  static const int kCopyVariants[] = {0, 1, 2, 3, 4, 5, 6, 7, 16, 17}, kMixVariants[] = {8, 9};
  const int *vs = mix ? kMixVariants : kCopyVariants;
  const int nv = mix ? 2 : 10;
  for (int j = 0; j < nv && !rc; j++) {
    const int v = vs[j];
    if (cog::launch_copy_peak(a, b, bytes, st, v)) rc = fail(COG_ERR_HIP, "copy launch failed");   // warm-up
    if (rc) break;
    (void)hipEventRecord(e0, st);
    for (int r = 0; r < iters && !rc; r++)
      if (cog::launch_copy_peak(a, b, bytes, st, v)) rc = fail(COG_ERR_HIP, "copy launch failed");
    (void)hipEventRecord(e1, st);
    float ms = 0.f;
    if (!rc && (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess))
      rc = fail(COG_ERR_HIP, "copy timing");
    if (!rc) best = std::max(best, (double)(bytes + out_bytes) * iters / ((double)ms * 1e-3) / 1e9);
  }
  if (!rc) *gb_per_s = best;
  if (st) (void)hipStreamSynchronize(st);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (st) (void)hipStreamDestroy(st);
  if (a) (void)hipFree(a);
  if (b) (void)hipFree(b);
  return rc;
}

void *cog_env_stream(cog_env *env) { return env ? (void *)env->sh[0].stream : nullptr; }
void *cog_env_shard_stream(cog_env *env, int k) {
  if (!env || k < 0 || (size_t)k >= env->sh.size()) return nullptr;
  return (void *)env->sh[k].stream;
}
int cog_env_device(const cog_env *env) { return env ? env->sh[0].device : -1; }

int cog_env_wait_stream(cog_env *env, int k, void *stream) {
  int rc = shard_of(env, k);
  if (rc) return rc;
  EnvShard &s = env->sh[k];
  DeviceGuard g(s.device);
  HIPCHK(hipEventRecord(s.ev, static_cast<hipStream_t>(stream)));
  HIPCHK(hipStreamWaitEvent(s.stream, s.ev, 0));
  return COG_OK;
}

int cog_env_signal_stream(cog_env *env, int k, void *stream) {
  int rc = shard_of(env, k);
  if (rc) return rc;
  EnvShard &s = env->sh[k];
  DeviceGuard g(s.device);
  HIPCHK(hipEventRecord(s.ev, s.stream));
  HIPCHK(hipStreamWaitEvent(static_cast<hipStream_t>(stream), s.ev, 0));
  return COG_OK;
}

int cog_env_invalidate_device(cog_env *env, void *stream) {
  if (!env) return fail(COG_ERR_INVALID, "env is NULL");
  int rc = prepare_host(env);
  if (rc) return rc;
  env_changed(env);                                        // (voids a speculative sample)
  for (EnvShard &k : env->sh) {
    DeviceGuard g(k.device);
    if (stream != COG_NO_STREAM) {                         // the caller's writes: order after them
      HIPCHK(hipEventRecord(k.ev, static_cast<hipStream_t>(stream)));
      HIPCHK(hipStreamWaitEvent(k.stream, k.ev, 0));
    }
    k.lean_clock = ~0ull;                                  // (edited masks or decks: any path)
    k.cdeck_ok = false;
    if (cog::launch_resync(k.s, k.stream))
      return fail(COG_ERR_HIP, std::string("resync launch failed: ") + hipGetErrorString(hipGetLastError()));
  }
  return finish(env, true);                                // (the host views, when there are any)
}

int cog_env_set_autoreset(cog_env *env, int on) {
  if (!env) return fail(COG_ERR_INVALID, "env is NULL");
  int rc = sync_all(env);
  if (rc) return rc;
  env_changed(env);
  for (EnvShard &k : env->sh) {
    k.s.autoreset = on ? 1u : 0u;
    k.lean_clock = ~0ull;
    k.cdeck_ok = false;
  }
  return COG_OK;
}

// ---- sampler -----------------------------------------------------------------------------
int cog_sampler_create_multi(size_t n_envs, uint64_t seed, const int *devices, int n_devices, cog_sampler **out) {
  return cog_sampler_create_at(n_envs, seed, 0, devices, n_devices, out);
}

int cog_sampler_create_at(size_t n_envs, uint64_t seed, uint64_t first_index, const int *devices, int n_devices,
                          cog_sampler **out) {
  if (!out) return fail(COG_ERR_INVALID, "out is NULL");
  *out = nullptr;
  int rc = check_devices(devices, n_devices);
  if (rc) return rc;
  cog_sampler *s = new cog_sampler();
  s->n = n_envs;
  if ((rc = zc_alloc(&s->h_actions, n_envs * COG_ACTION_BYTES))) {
    sampler_free(s);
    return rc;
  }
  std::memset(s->h_actions, 0, n_envs * COG_ACTION_BYTES);
  if ((rc = hmalloc(&s->h_sig, 256 * (size_t)n_devices, hipHostMallocMapped | hipHostMallocCoherent))) {
    sampler_free(s);
    return rc;
  }
  std::memset(s->h_sig, 0, 256 * (size_t)n_devices);
  const std::vector<size_t> first = block_split(n_envs, n_devices);
  s->sh.resize(n_devices);
  for (int j = 0; j < n_devices; j++) {
    SamplerShard &k = s->sh[j];
    k.device = devices[j];
    k.first = first[j];
    k.n = first[j + 1] - first[j];
    DeviceGuard g(k.device);
    if (hipStreamCreateWithFlags(&k.stream, hipStreamNonBlocking) != hipSuccess) {
      sampler_free(s);
      return fail(COG_ERR_HIP, "hipStreamCreate failed");
    }
    if ((rc = dmalloc(&k.d_rng, k.n * sizeof(uint32_t))) || (rc = dmalloc(&k.d_actions, k.n * COG_ACTION_BYTES)) ||
        (rc = dmalloc(&k.d_masks, k.n * COG_MASK_BYTES)) || (rc = dmalloc(&k.done.ctr, 256))) {
      sampler_free(s);
      return rc;
    }
    void *d_sig = nullptr;
    if (hipHostGetDevicePointer(&d_sig, s->h_sig + 64 * j, 0) == hipSuccess) {
      k.done.h = s->h_sig + 64 * j;
      k.done.d = static_cast<uint32_t *>(d_sig);
    }
    // vec_action_sampler(seed) (vec_sampler.h:9-13): sampler i seeded seed + i, seed a u32, the sum
    // in size_t; i is the global index first_index + k.first + j
    if (hipMemsetAsync(k.d_actions, 0, k.n * COG_ACTION_BYTES, k.stream) != hipSuccess ||
        hipMemsetAsync(k.done.ctr, 0, 256, k.stream) != hipSuccess ||
        cog::launch_seed_sampler(k.n, (uint64_t)(uint32_t)seed, (size_t)first_index + k.first, k.d_rng, k.stream)) {
      sampler_free(s);
      return fail(COG_ERR_HIP, "sampler init failed");
    }
  }
  for (SamplerShard &k : s->sh) {
    DeviceGuard g(k.device);
    if (hipStreamSynchronize(k.stream) != hipSuccess) {
      sampler_free(s);
      return fail(COG_ERR_HIP, "sampler init failed");
    }
  }
  sampler_register(s, true);
  *out = s;
  return COG_OK;
}

int cog_sampler_create(size_t n_envs, uint64_t seed, int device, cog_sampler **out) {
  return cog_sampler_create_multi(n_envs, seed, &device, 1, out);
}

void cog_sampler_destroy(cog_sampler *s) { sampler_free(s); }

int cog_sampler_num_shards(const cog_sampler *s, int *out) {
  if (!s || !out) return fail(COG_ERR_INVALID, "NULL argument");
  *out = (int)s->sh.size();
  return COG_OK;
}

// signal: the sampler kernel stores the shard's completion word (host calls on the sampler's
// own stream)
static int sampler_run(SamplerShard &k, cog_action_t *h_actions, const uint8_t *d_masks, hipStream_t stream,
                       bool host_refresh, bool signal = false) {
  uint8_t *h_act = host_refresh && k.n ? const_cast<uint8_t *>(zc_device(h_actions + k.first, k.n * COG_ACTION_BYTES)) : nullptr;
  if (h_act && !zc_same_on(k.device, h_actions)) h_act = nullptr;
  uint32_t seq = 0;
  uint32_t *ctr = signal && h_act ? signal_arm(k.done, seq) : nullptr;
  if (cog::launch_sample(k.n, d_masks, k.d_rng, k.d_actions, stream, h_act, ctr, k.done.d, seq))   // actions to the host view in place
    return fail(COG_ERR_HIP, std::string("sample launch failed: ") + hipGetErrorString(hipGetLastError()));
  if (ctr) signal_armed(k.done);
  if (host_refresh && k.n && !h_act)
    HIPCHK(hipMemcpyAsync(h_actions + k.first, k.d_actions, k.n * COG_ACTION_BYTES, hipMemcpyDeviceToHost, stream));
  return COG_OK;
}

int cog_sampler_sample_device(cog_sampler *s, const void *d_masks, size_t n) {
  if (!s || !d_masks) return fail(COG_ERR_INVALID, "NULL argument");
  if (n != s->n) return fail(COG_ERR_INVALID, "action_mask length != num_envs");
  s->version++;
  if (s->sh.size() != 1) return fail(COG_ERR_INVALID, "device masks need a single-shard sampler (one device pointer)");
  SamplerShard &k = s->sh[0];
  DeviceGuard g(k.device);
  k.done.queued = false;
  int rc = sampler_run(k, s->h_actions, static_cast<const uint8_t *>(d_masks), k.stream, true, true);
  if (rc || (rc = signal_enqueue(k.done, k.stream))) return rc;
  return signal_wait(k.done, k.stream);
}

int cog_sampler_sample(cog_sampler *s, const cog_action_mask_t *masks, size_t n) {
  if (!s || (!masks && n)) return fail(COG_ERR_INVALID, "NULL argument");
  if (n != s->n) return fail(COG_ERR_INVALID, "action_mask length != num_envs");
  SamplerSpec &sp = s->spec;
  const bool hit = sp.ok && sp.version == s->version && sp.env && env_alive(sp.env) && single(sp.env) &&
                   masks == sp.env->h_sel && sp.env->n == n && sp.env->version == sp.env_version &&
                   *reinterpret_cast<volatile uint32_t *>(sp.h + n * 8) == 0u;
  sp.ok = false;
  s->version++;
  if (hit) {                                               // the env's step sampled these masks already
    SamplerShard &k = s->sh[0];
    std::swap(k.d_rng, sp.d_rng);
    std::swap(k.d_actions, sp.d_actions);
    const uint64_t *src = reinterpret_cast<const uint64_t *>(sp.h);
    uint8_t *dst = reinterpret_cast<uint8_t *>(s->h_actions);
    for (size_t i = 0; i < n; i++) *reinterpret_cast<uint64_t *>(dst + i * COG_ACTION_BYTES) = src[i];
    s->spec_hits++;
    return COG_OK;
  }
  for (SamplerShard &k : s->sh) k.done.queued = false;
  for (SamplerShard &k : s->sh) {
    if (!k.n) continue;
    DeviceGuard g(k.device);
    const uint8_t *dm = nullptr;
    if (EnvShard *ek = env_masks_in_hbm(masks + k.first, k.n, k.device)) {    // an env's own view: HBM
      if (env_stream_in_flight(*ek)) {                     // the sampler's stream after the env's step
        HIPCHK(hipEventRecord(ek->ev, ek->stream));
        HIPCHK(hipStreamWaitEvent(k.stream, ek->ev, 0));
      }
      dm = ek->s.sel;
    }
    if (!dm) {
      dm = zc_device(masks + k.first, k.n * COG_MASK_BYTES);                // else read in place when pinned
      if (!dm || !zc_same_on(k.device, masks + k.first)) {
        HIPCHK(hipMemcpyAsync(k.d_masks, masks + k.first, k.n * COG_MASK_BYTES, hipMemcpyHostToDevice, k.stream));
        dm = k.d_masks;
      }
    }
    int rc = sampler_run(k, s->h_actions, dm, k.stream, true, true);
    if (rc || (rc = signal_enqueue(k.done, k.stream))) return rc;
  }
  for (SamplerShard &k : s->sh) {
    DeviceGuard g(k.device);
    int rc = signal_wait(k.done, k.stream);
    if (rc) return rc;
  }
  return COG_OK;
}

cog_action_t *cog_sampler_actions(cog_sampler *s) { return s ? s->h_actions : nullptr; }
void *cog_sampler_device_actions(cog_sampler *s) {
  if (!s) return nullptr;
  s->exported = true;                                      // (aliases: no buffer swaps from now on)
  return (void *)s->sh[0].d_actions;
}
void *cog_sampler_shard_device_actions(cog_sampler *s, int k) {
  if (!s || k < 0 || (size_t)k >= s->sh.size()) return nullptr;
  s->exported = true;
  return (void *)s->sh[k].d_actions;
}
int cog_sampler_device(const cog_sampler *s) { return s ? s->sh[0].device : -1; }
int cog_sampler_spec_stats(const cog_sampler *s, uint64_t *samples, uint64_t *hits) {
  if (!s || !samples || !hits) return fail(COG_ERR_INVALID, "NULL argument");
  *samples = s->version;
  *hits = s->spec_hits;
  return COG_OK;
}

// ---- runner ------------------------------------------------------------------------------
int cog_runner_create(cog_env *env, cog_sampler *s, size_t n_threads, uint32_t flags, cog_runner **out) {
  if (!env || !s || !out) return fail(COG_ERR_INVALID, "NULL argument");
  if (env->n != s->n) return fail(COG_ERR_INVALID, "env and sampler batch sizes differ");
  if (env->sh.size() != s->sh.size()) return fail(COG_ERR_INVALID, "env and sampler are sharded differently");
  for (size_t j = 0; j < env->sh.size(); j++)
    if (env->sh[j].device != s->sh[j].device || env->sh[j].first != s->sh[j].first || env->sh[j].n != s->sh[j].n)
      return fail(COG_ERR_INVALID, "env and sampler are on different devices");
  cog_runner *r = new cog_runner();
  r->env = env;
  r->smp = s;
  r->n_threads = n_threads;
  r->flags = flags;
  r->ev.resize(env->sh.size());
  const char *cv = std::getenv("COG_RUNNER_CHUNK");        // default rollout steps per launch
  r->chunk = cv ? std::max(1, std::atoi(cv)) : 1;
  *out = r;
  return COG_OK;
}

void cog_runner_destroy(cog_runner *r) {
  if (!r) return;
  for (size_t j = 0; j < r->env->sh.size(); j++) {
    DeviceGuard g(r->env->sh[j].device);
    (void)hipStreamSynchronize(r->env->sh[j].stream);
    for (hipEvent_t ev : r->ev[j]) (void)hipEventDestroy(ev);
  }
  delete r;
}

size_t cog_runner_n_threads(const cog_runner *r) { return r ? r->n_threads : 0; }

static bool runner_host(const cog_runner *r) { return !(r->flags & COG_RUNNER_DEVICE_VIEWS) && r->env->host; }

static int runner_flush_sample(cog_runner *r) {
  if (!r->pending_sample) return COG_OK;
  r->pending_sample = false;
  r->smp->version++;
  // a lone sample reads the selected masks, as the reference runner's does (runner.h:26,48);
  // stored-mask sampling exists only fused with a step
  for (size_t j = 0; j < r->env->sh.size(); j++) {
    EnvShard &k = r->env->sh[j];
    DeviceGuard g(k.device);
    if (k.pub_done) {                                      // the actions' view needs the next publish
      k.pub_done = false;
      k.done.queued = false;
    }
    int rc = sampler_run(r->smp->sh[j], r->smp->h_actions, k.s.sel, k.stream, false);
    if (rc) return rc;
  }
  return COG_OK;
}

static int runner_timing_event(cog_runner *r, size_t j) {
  std::vector<hipEvent_t> &v = r->ev[j];
  while (r->ev_used + 1 >= v.size()) {
    hipEvent_t ev;
    HIPCHK(hipEventCreate(&ev));
    v.push_back(ev);
  }
  return COG_OK;
}

// `steps` fused sample+step launches on every shard; with timing on, one event pair per shard
// brackets the batch (device time per launch = pair time / steps, the quantity rocprofv3's
// kernel trace averages, without per-launch event overhead)
// A shard's host-visible work that is not a direct publish: the views are stale until the next
// publish, and a completion word armed by an earlier direct step no longer covers the stream.
static void views_pending(EnvShard &k) {
  k.host_synced = false;
  k.pub_done = false;
  k.done.queued = false;
}

static int runner_launch_fused(cog_runner *r, int steps) {
  const int src = (r->flags & COG_RUNNER_STORED_MASKS) ? cog::MASK_STORED : cog::MASK_SELECTED;
  env_changed(r->env);
  r->smp->version++;
  const bool host = runner_host(r);
  int rc;
  if (host && (rc = prepare_host(r->env))) return rc;
  for (size_t j = 0; j < r->env->sh.size(); j++) {
    EnvShard &k = r->env->sh[j];
    SamplerShard &q = r->smp->sh[j];
    DeviceGuard g(k.device);
    // one host-visible step with the views in sync (runner.sample(); runner.step()): the step
    // publishes itself, the sampled actions included (k_env_step_pub), as env.step() does
    if (host && steps == 1 && !r->timing && k.zc && k.mir_valid && k.host_synced && cog::step_pub_ok(k.n) && q.n) {
      k.lean_clock = ~0ull;                                // (a full step: not the trio)
      k.cdeck_ok = false;
      uint8_t *h_act = const_cast<uint8_t *>(zc_device(r->smp->h_actions + q.first, q.n * COG_ACTION_BYTES));
      uint32_t seq = 0, *ctr = nullptr;
      if (h_act && zc_same_on(k.device, r->smp->h_actions + q.first) && (ctr = signal_arm(k.done, seq))) {
        cog::DevState ps = launch_state(k, true);
        ps.pub_obs = k.h_obs_d;
        ps.pub_outs = k.h_outs_d;
        ps.pub_mir = k.mir;
        if (cog::launch_sample_step_pub(ps, src, q.d_rng, q.d_actions, h_act, k.stream, ctr, k.done.d, seq))
          return fail(COG_ERR_HIP, std::string("sample_step launch failed: ") + hipGetErrorString(hipGetLastError()));
        signal_armed(k.done);
        k.pub_done = true;                                 // (host_synced stays: the step keeps the views)
        continue;
      }
    }
    views_pending(k);                                      // (device work: views stale until a publish)
    if (r->timing) {
      if ((rc = runner_timing_event(r, j))) return rc;
      HIPCHK(hipEventRecord(r->ev[j][r->ev_used], k.stream));
    }
    const cog::DevState s = launch_state(k, host);
    if (r->chunk > 1) {                                    // persistent kernels, chunk steps each
      const bool trio = cog::rollout_kind_of(k.n, src, r->env->n_players >= 3) == 3;
      for (int t = 0; t < steps; t += r->chunk) {
        const int kk = std::min(r->chunk, steps - t);
        // no env can park in this launch (EnvShard::lean_clock): no fix-up launch
        const bool no_fixup = trio && k.s.autoreset && k.lean_clock != ~0ull &&
                              k.lean_clock + (uint64_t)kk < (uint64_t)r->env->max_steps;
        cog::DevState sc = s;
        sc.cdeck_ok = trio && k.cdeck_ok ? 1u : 0u;
#ifdef COG_NO_CDECK                                        // (A/B probe builds: the DeckObs loads always)
        sc.cdeck_ok = 0u;
#endif
        if (cog::launch_rollout(sc, src, kk, q.d_rng, q.d_actions, k.stream, r->env->n_players >= 3, &k.park_seq,
                                no_fixup))
          return fail(COG_ERR_HIP, std::string("rollout launch failed: ") + hipGetErrorString(hipGetLastError()));
        k.lean_clock = trio && k.lean_clock != ~0ull ? k.lean_clock + (uint64_t)kk : ~0ull;
        k.cdeck_ok = trio;                                 // (the trio and its fix-up write cdeck)
      }
    } else {
      k.lean_clock = ~0ull;                                // (full steps)
      k.cdeck_ok = false;
      for (int t = 0; t < steps; t++)
        if (cog::launch_sample_step(s, src, q.d_rng, q.d_actions, k.stream))
          return fail(COG_ERR_HIP, std::string("sample_step launch failed: ") + hipGetErrorString(hipGetLastError()));
    }
    if (r->timing) HIPCHK(hipEventRecord(r->ev[j][r->ev_used + 1], k.stream));
  }
  if (r->timing) {
    r->ev_used += 2;
    r->timed_launches += (uint64_t)steps;
  }
  return COG_OK;
}

int cog_runner_sample(cog_runner *r) {
  if (!r) return fail(COG_ERR_INVALID, "runner is NULL");
  int rc = runner_flush_sample(r);   // two samples in a row: the first one still runs
  if (rc) return rc;
  r->pending_sample = true;
  return COG_OK;
}

int cog_runner_step(cog_runner *r) {
  if (!r) return fail(COG_ERR_INVALID, "runner is NULL");
  env_changed(r->env);
  if (r->pending_sample) {
    r->pending_sample = false;
    return runner_launch_fused(r, 1);
  }
  const bool host = runner_host(r);
  int rc;
  if (host && (rc = prepare_host(r->env))) return rc;
  for (EnvShard &k : r->env->sh) views_pending(k);
  for (size_t j = 0; j < r->env->sh.size(); j++) {
    EnvShard &k = r->env->sh[j];
    DeviceGuard g(k.device);
    k.lean_clock = ~0ull;                                  // (a full step)
    k.cdeck_ok = false;
    if (cog::launch_step(launch_state(k, host), r->smp->sh[j].d_actions, k.stream))
      return fail(COG_ERR_HIP, std::string("step launch failed: ") + hipGetErrorString(hipGetLastError()));
  }
  return COG_OK;
}

int cog_runner_rollout(cog_runner *r, int steps) {
  if (!r || steps < 0) return fail(COG_ERR_INVALID, "bad argument");
  int rc = runner_flush_sample(r);
  if (rc) return rc;
  return steps ? runner_launch_fused(r, steps) : COG_OK;
}

int cog_runner_sync(cog_runner *r) {
  if (!r) return fail(COG_ERR_INVALID, "runner is NULL");
  int rc = runner_flush_sample(r);
  if (rc) return rc;
  const bool host = !(r->flags & COG_RUNNER_DEVICE_VIEWS);
  if (host && !r->env->host) {                       // no env views yet: the sampler's view alone
    for (size_t j = 0; j < r->env->sh.size(); j++) {
      EnvShard &k = r->env->sh[j];
      SamplerShard &q = r->smp->sh[j];
      if (!q.n) continue;
      DeviceGuard g(k.device);
      HIPCHK(hipMemcpyAsync(r->smp->h_actions + q.first, q.d_actions, q.n * COG_ACTION_BYTES, hipMemcpyDeviceToHost,
                            k.stream));
    }
  }
  return finish(r->env, host, host && r->env->host ? r->smp : nullptr);   // (the actions ride with the env's views)
}

int cog_runner_set_chunk(cog_runner *r, int steps_per_launch) {
  if (!r || steps_per_launch < 1) return fail(COG_ERR_INVALID, "bad argument");
  r->chunk = steps_per_launch;
  return COG_OK;
}

int cog_runner_set_timing(cog_runner *r, int enable) {
  if (!r) return fail(COG_ERR_INVALID, "runner is NULL");
  r->timing = enable != 0;
  r->ev_used = 0;
  r->timed_launches = 0;
  return COG_OK;
}

// device time: per shard the sum over its event pairs; the slowest shard's total
int cog_runner_kernel_time(cog_runner *r, double *total_ms, uint64_t *launches) {
  if (!r) return fail(COG_ERR_INVALID, "runner is NULL");
  int rc = sync_all(r->env);
  if (rc) return rc;
  double worst = 0.0;
  for (size_t j = 0; j < r->env->sh.size(); j++) {
    double acc = 0.0;
    for (size_t q = 0; q + 1 < r->ev_used && q + 1 < r->ev[j].size(); q += 2) {
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, r->ev[j][q], r->ev[j][q + 1]));
      acc += ms;
    }
    worst = std::max(worst, acc);
  }
  if (total_ms) *total_ms = worst;
  if (launches) *launches = r->timed_launches;
  r->ev_used = 0;
  r->timed_launches = 0;
  return COG_OK;
}

}  // extern "C"
