// cog_abi.cpp -- host side of libcog_hip.so: implements the C ABI of include/cog.h on top of the
// kernels in cog_engine.hip.  Owns device buffers, the per-handle HIP stream, the lazily
// allocated pinned host views and the asynchronous runner.  No CPU fallback exists: without a
// gfx950 device every constructor fails with COG_ERR_NODEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
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
int hmalloc(T **p, size_t bytes) {
  if (hipHostMalloc(reinterpret_cast<void **>(p), bytes ? bytes : 64, hipHostMallocDefault) != hipSuccess)
    return fail(COG_ERR_OOM, "hipHostMalloc of " + std::to_string(bytes) + " bytes failed");
  return COG_OK;
}

}  // namespace

struct cog_env {
  int device = 0;
  hipStream_t stream = nullptr;
  cog::DevState s{};
  uint8_t *d_actions = nullptr;       // staging for host-provided actions
  // pinned host views (lazy)
  bool host = false;
  cog_obs_t *h_obs = nullptr;
  cog_action_mask_t *h_sel = nullptr;
  float *h_rew = nullptr;
  uint8_t *h_done = nullptr;
  uint8_t *h_agent = nullptr;
  cog_info_t *h_info = nullptr;
  uint32_t *h_status = nullptr;       // pinned [4]
  std::vector<uint32_t> dirty;
};

struct cog_sampler {
  int device = 0;
  hipStream_t stream = nullptr;
  size_t n = 0;
  uint32_t *d_rng = nullptr;
  uint8_t *d_actions = nullptr;
  uint8_t *d_masks = nullptr;         // staging for host-provided masks
  cog_action_t *h_actions = nullptr;
};

struct cog_runner {
  cog_env *env = nullptr;
  cog_sampler *smp = nullptr;
  size_t n_threads = 0;
  uint32_t flags = 0;
  bool pending_sample = false;
  bool timing = false;
  std::vector<hipEvent_t> ev;         // pairs: one per step() launch or one per rollout() batch
  size_t ev_used = 0;
  uint64_t timed_launches = 0;        // fused launches covered by the recorded pairs
  int chunk = 1;                      // rollout steps per launch (>1: persistent K-step kernel)
};

namespace {

void env_free(cog_env *e) {
  if (!e) return;
  DeviceGuard g(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  void *dev[] = {e->s.obs, e->s.sel, e->s.info, e->s.rew, e->s.done, e->s.agent, e->s.priv,
                 e->s.grid, e->s.cgrid, e->s.heads, e->s.park, e->s.gen, e->s.status, e->s.dirty, e->d_actions};
  for (void *p : dev)
    if (p) (void)hipFree(p);
  void *hst[] = {e->h_obs, e->h_sel, e->h_rew, e->h_done, e->h_agent, e->h_info, e->h_status};
  for (void *p : hst)
    if (p) (void)hipHostFree(p);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

int read_status(cog_env *e, uint32_t out[4]) {
  HIPCHK(hipMemcpyAsync(e->h_status, e->s.status, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  std::memcpy(out, e->h_status, 4 * sizeof(uint32_t));
  HIPCHK(hipMemsetAsync(e->s.status, 0, 4 * sizeof(uint32_t), e->stream));
  return COG_OK;
}

int status_to_rc(const uint32_t st[4]) {
  if (st[1]) {
    if (st[0] & cog::F_GRID_OVER)
      return fail(COG_ERR_MAPGEN, "map generation produced a map larger than the 48x48 observation grid");
    return fail(COG_ERR_MAPGEN, "Failed to generate map in specified maximum number of attempts");
  }
  return COG_OK;
}

// enqueue D2H of everything a step can change (obs dynamic tail, masks, outputs)
int enqueue_refresh_tail(cog_env *e) {
  const size_t n = e->s.n;
  if (!n) return COG_OK;
  HIPCHK(hipMemcpy2DAsync(reinterpret_cast<uint8_t *>(e->h_obs) + COG_OBS_MAP_BYTES, COG_OBS_BYTES,
                          e->s.obs + COG_OBS_MAP_BYTES, COG_OBS_BYTES, COG_OBS_BYTES - COG_OBS_MAP_BYTES,
                          n, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(e->h_sel, e->s.sel, n * COG_MASK_BYTES, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(e->h_rew, e->s.rew, n * 4 * sizeof(float), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(e->h_done, e->s.done, n, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(e->h_agent, e->s.agent, n, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(e->h_info, e->s.info, n * COG_INFO_BYTES, hipMemcpyDeviceToHost, e->stream));
  return COG_OK;
}

int refresh_full(cog_env *e) {
  if (!e->host || !e->s.n) return COG_OK;
  HIPCHK(hipMemcpyAsync(e->h_obs, e->s.obs, e->s.n * COG_OBS_BYTES, hipMemcpyDeviceToHost, e->stream));
  int rc = enqueue_refresh_tail(e);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(e->stream));
  return COG_OK;
}

// after steps: status word + dynamic tail, then the maps of re-generated envs
int finish_steps(cog_env *e, bool refresh_host) {
  if (refresh_host && e->host) {
    int rc = enqueue_refresh_tail(e);
    if (rc) return rc;
  }
  uint32_t st[4];
  int rc = read_status(e, st);
  if (rc) return rc;
  const uint32_t ndirty = st[2];
  if (refresh_host && e->host && ndirty) {
    if (ndirty >= e->s.n / 8) {   // many resets (or list overflow): copy every map
      HIPCHK(hipMemcpy2DAsync(e->h_obs, COG_OBS_BYTES, e->s.obs, COG_OBS_BYTES, COG_OBS_MAP_BYTES, e->s.n,
                              hipMemcpyDeviceToHost, e->stream));
    } else {
      e->dirty.resize(ndirty);
      HIPCHK(hipMemcpy(e->dirty.data(), e->s.dirty, ndirty * sizeof(uint32_t), hipMemcpyDeviceToHost));
      for (uint32_t k = 0; k < ndirty; k++) {
        const size_t i = e->dirty[k];
        HIPCHK(hipMemcpyAsync(reinterpret_cast<uint8_t *>(e->h_obs) + i * COG_OBS_BYTES,
                              e->s.obs + i * COG_OBS_BYTES, COG_OBS_MAP_BYTES, hipMemcpyDeviceToHost, e->stream));
      }
    }
    HIPCHK(hipStreamSynchronize(e->stream));
  }
  return status_to_rc(st);
}

void sampler_free(cog_sampler *s) {
  if (!s) return;
  DeviceGuard g(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  void *dev[] = {s->d_rng, s->d_actions, s->d_masks};
  for (void *p : dev)
    if (p) (void)hipFree(p);
  if (s->h_actions) (void)hipHostFree(s->h_actions);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

}  // namespace

extern "C" {

const char *cog_last_error(void) { return g_err.c_str(); }
int cog_abi_version(void) { return COG_ABI_VERSION; }

int cog_device_count(int *out) {
  if (!out) return fail(COG_ERR_INVALID, "out is NULL");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *out = n;
  return COG_OK;
}

int cog_env_create(size_t n_envs, int device, cog_env **out) {
  if (!out) return fail(COG_ERR_INVALID, "out is NULL");
  *out = nullptr;
  int rc = check_device(device);
  if (rc) return rc;
  DeviceGuard g(device);
  cog_env *e = new cog_env();
  e->device = device;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
    env_free(e);
    return fail(COG_ERR_HIP, "hipStreamCreate failed");
  }
  const size_t n = n_envs;
  cog::DevState &s = e->s;
  s.n = n;
  s.first = 0;
  s.cap = n;
  s.autoreset = 1;
  if ((rc = dmalloc(&s.obs, n * COG_OBS_BYTES)) || (rc = dmalloc(&s.sel, n * COG_MASK_BYTES)) ||
      (rc = dmalloc(&s.info, n * COG_INFO_BYTES)) || (rc = dmalloc(&s.rew, n * 4 * sizeof(float))) ||
      (rc = dmalloc(&s.done, n)) || (rc = dmalloc(&s.agent, n)) ||
      (rc = dmalloc(&s.priv, n * sizeof(cog::EnvPriv))) ||
      (rc = dmalloc(&s.grid, n * (size_t)cog::kGridBytes)) || (rc = dmalloc(&s.cgrid, n * (size_t)COG_CELLS)) ||
      (rc = dmalloc(&s.heads, n * 5 * sizeof(uint4))) || (rc = dmalloc(&s.park, n * sizeof(uint32_t))) ||
      (rc = dmalloc(&s.gen, n * sizeof(cog::GenScratch))) || (rc = dmalloc(&s.status, 64)) ||
      (rc = dmalloc(&s.dirty, n * sizeof(uint32_t))) || (rc = dmalloc(&e->d_actions, n * COG_ACTION_BYTES)) ||
      (rc = hmalloc(&e->h_status, 64))) {
    env_free(e);
    return rc;
  }
  struct { void *p; size_t b; } z[] = {
      {s.obs, n * COG_OBS_BYTES}, {s.sel, n * COG_MASK_BYTES}, {s.info, n * COG_INFO_BYTES},
      {s.rew, n * 4 * sizeof(float)}, {s.done, n}, {s.agent, n}, {s.grid, n * (size_t)cog::kGridBytes},
      {s.cgrid, n * (size_t)COG_CELLS},
      {s.gen, n * sizeof(cog::GenScratch)}, {s.status, 64}, {e->d_actions, n * COG_ACTION_BYTES}};
  for (auto &zz : z)
    if (zz.b && hipMemsetAsync(zz.p, 0, zz.b, e->stream) != hipSuccess) {
      env_free(e);
      return fail(COG_ERR_HIP, "hipMemsetAsync failed");
    }
  if (hipMemsetAsync(s.park, 0xff, n * sizeof(uint32_t), e->stream) != hipSuccess) {   // nothing parked
    env_free(e);
    return fail(COG_ERR_HIP, "hipMemsetAsync failed");
  }
  const uint32_t default_seed = std::random_device{}();   // cog_env() seeds from random_device
  if (cog::launch_init(s, nullptr, default_seed, e->stream) || hipStreamSynchronize(e->stream) != hipSuccess) {
    env_free(e);
    return fail(COG_ERR_HIP, std::string("env init kernel failed: ") + hipGetErrorString(hipGetLastError()));
  }
  *out = e;
  return COG_OK;
}

void cog_env_destroy(cog_env *env) { env_free(env); }

int cog_env_num_envs(const cog_env *env, size_t *out) {
  if (!env || !out) return fail(COG_ERR_INVALID, "NULL argument");
  *out = env->s.n;
  return COG_OK;
}

static int env_reset_impl(cog_env *e, const cog::ResetParams &p) {
  DeviceGuard g(e->device);
  if (cog::launch_reset(e->s, p, e->stream) || cog::launch_encode_all(e->s, e->stream))
    return fail(COG_ERR_HIP, std::string("reset launch failed: ") + hipGetErrorString(hipGetLastError()));
  uint32_t st[4];
  int rc = read_status(e, st);
  if (rc) return rc;
  rc = refresh_full(e);
  if (rc) return rc;
  return status_to_rc(st);
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

int cog_env_step_device(cog_env *env, const void *d_actions, size_t n) {
  if (!env || !d_actions) return fail(COG_ERR_INVALID, "NULL argument");
  if (n != env->s.n) return fail(COG_ERR_INVALID, "actions length != num_envs");
  DeviceGuard g(env->device);
  if (cog::launch_step(env->s, static_cast<const uint8_t *>(d_actions), env->stream))
    return fail(COG_ERR_HIP, std::string("step launch failed: ") + hipGetErrorString(hipGetLastError()));
  return finish_steps(env, true);
}

int cog_env_step(cog_env *env, const cog_action_t *actions, size_t n) {
  if (!env || (!actions && n)) return fail(COG_ERR_INVALID, "NULL argument");
  if (n != env->s.n) return fail(COG_ERR_INVALID, "actions length != num_envs");
  DeviceGuard g(env->device);
  if (n) HIPCHK(hipMemcpyAsync(env->d_actions, actions, n * COG_ACTION_BYTES, hipMemcpyHostToDevice, env->stream));
  return cog_env_step_device(env, env->d_actions, n);
}

int cog_env_get_views(cog_env *env, cog_env_views *out) {
  if (!env || !out) return fail(COG_ERR_INVALID, "NULL argument");
  DeviceGuard g(env->device);
  if (!env->host) {
    const size_t n = env->s.n;
    int rc;
    if ((rc = hmalloc(&env->h_obs, n * COG_OBS_BYTES)) || (rc = hmalloc(&env->h_sel, n * COG_MASK_BYTES)) ||
        (rc = hmalloc(&env->h_rew, n * 4 * sizeof(float))) || (rc = hmalloc(&env->h_done, n)) ||
        (rc = hmalloc(&env->h_agent, n)) || (rc = hmalloc(&env->h_info, n * COG_INFO_BYTES)))
      return rc;
    std::memset(env->h_obs, 0, n * COG_OBS_BYTES);   // padding bytes stay defined
    env->host = true;
    rc = refresh_full(env);
    if (rc) return rc;
  }
  out->n_envs = env->s.n;
  out->observations = env->h_obs;
  out->selected_action_masks = env->h_sel;
  out->rewards = env->h_rew;
  out->dones = env->h_done;
  out->agent_selection = env->h_agent;
  out->infos = env->h_info;
  out->d_observations = env->s.obs;
  out->d_selected_action_masks = env->s.sel;
  out->d_rewards = env->s.rew;
  out->d_dones = env->s.done;
  out->d_agent_selection = env->s.agent;
  out->d_infos = env->s.info;
  return COG_OK;
}

int cog_env_sync_host(cog_env *env) {
  if (!env) return fail(COG_ERR_INVALID, "env is NULL");
  DeviceGuard g(env->device);
  return refresh_full(env);
}

int cog_env_hazards(cog_env *env, uint32_t *flags_or, uint32_t *per_env) {
  if (!env) return fail(COG_ERR_INVALID, "env is NULL");
  DeviceGuard g(env->device);
  std::vector<uint32_t> tmp(env->s.n);
  if (env->s.n)
    HIPCHK(hipMemcpy2DAsync(tmp.data(), sizeof(uint32_t), reinterpret_cast<uint8_t *>(env->s.priv) + offsetof(cog::EnvPriv, flags),
                            sizeof(cog::EnvPriv), sizeof(uint32_t), env->s.n, hipMemcpyDeviceToHost, env->stream));
  HIPCHK(hipStreamSynchronize(env->stream));
  uint32_t acc = 0;
  for (uint32_t f : tmp) acc |= f;
  if (flags_or) *flags_or = acc;
  if (per_env) std::memcpy(per_env, tmp.data(), tmp.size() * sizeof(uint32_t));
  return COG_OK;
}

int cog_env_clear_hazards(cog_env *env) {
  if (!env) return fail(COG_ERR_INVALID, "env is NULL");
  DeviceGuard g(env->device);
  if (env->s.n)
    HIPCHK(hipMemset2DAsync(reinterpret_cast<uint8_t *>(env->s.priv) + offsetof(cog::EnvPriv, flags), sizeof(cog::EnvPriv),
                            0, sizeof(uint32_t), env->s.n, env->stream));
  HIPCHK(hipStreamSynchronize(env->stream));
  return COG_OK;
}

int cog_env_time_encode(cog_env *env, int iters, int variant, double *ms_per_launch) {
  if (!env || iters < 1 || !ms_per_launch) return fail(COG_ERR_INVALID, "bad argument");
  DeviceGuard g(env->device);
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  if (cog::launch_encode_all(env->s, env->stream, variant))   // warm-up launch
    return fail(COG_ERR_HIP, "encode launch failed");
  HIPCHK(hipEventRecord(e0, env->stream));
  for (int k = 0; k < iters; k++)
    if (cog::launch_encode_all(env->s, env->stream, variant)) return fail(COG_ERR_HIP, "encode launch failed");
  HIPCHK(hipEventRecord(e1, env->stream));
  HIPCHK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  *ms_per_launch = (double)ms / iters;
  return COG_OK;
}

void *cog_env_stream(cog_env *env) { return env ? (void *)env->stream : nullptr; }
int cog_env_device(const cog_env *env) { return env ? env->device : -1; }
int cog_env_set_autoreset(cog_env *env, int on) {
  if (!env) return fail(COG_ERR_INVALID, "env is NULL");
  DeviceGuard g(env->device);
  if (hipStreamSynchronize(env->stream) != hipSuccess) return fail(COG_ERR_HIP, "hipStreamSynchronize failed");
  env->s.autoreset = on ? 1u : 0u;
  return COG_OK;
}
int cog_sampler_device(const cog_sampler *s) { return s ? s->device : -1; }

// ---- sampler -----------------------------------------------------------------------------
int cog_sampler_create(size_t n_envs, uint64_t seed, int device, cog_sampler **out) {
  if (!out) return fail(COG_ERR_INVALID, "out is NULL");
  *out = nullptr;
  int rc = check_device(device);
  if (rc) return rc;
  DeviceGuard g(device);
  cog_sampler *s = new cog_sampler();
  s->device = device;
  s->n = n_envs;
  if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
    sampler_free(s);
    return fail(COG_ERR_HIP, "hipStreamCreate failed");
  }
  if ((rc = dmalloc(&s->d_rng, n_envs * sizeof(uint32_t))) || (rc = dmalloc(&s->d_actions, n_envs * COG_ACTION_BYTES)) ||
      (rc = dmalloc(&s->d_masks, n_envs * COG_MASK_BYTES)) || (rc = hmalloc(&s->h_actions, n_envs * COG_ACTION_BYTES))) {
    sampler_free(s);
    return rc;
  }
  std::memset(s->h_actions, 0, n_envs * COG_ACTION_BYTES);
  if (hipMemsetAsync(s->d_actions, 0, n_envs * COG_ACTION_BYTES, s->stream) != hipSuccess ||
      cog::launch_seed_sampler(n_envs, (uint32_t)seed, s->d_rng, s->stream) ||
      hipStreamSynchronize(s->stream) != hipSuccess) {
    sampler_free(s);
    return fail(COG_ERR_HIP, "sampler init failed");
  }
  *out = s;
  return COG_OK;
}

void cog_sampler_destroy(cog_sampler *s) { sampler_free(s); }

static int sampler_run(cog_sampler *s, const uint8_t *d_masks, hipStream_t stream, bool host_refresh) {
  if (cog::launch_sample(s->n, d_masks, s->d_rng, s->d_actions, stream))
    return fail(COG_ERR_HIP, std::string("sample launch failed: ") + hipGetErrorString(hipGetLastError()));
  if (host_refresh && s->n)
    HIPCHK(hipMemcpyAsync(s->h_actions, s->d_actions, s->n * COG_ACTION_BYTES, hipMemcpyDeviceToHost, stream));
  return COG_OK;
}

int cog_sampler_sample_device(cog_sampler *s, const void *d_masks, size_t n) {
  if (!s || !d_masks) return fail(COG_ERR_INVALID, "NULL argument");
  if (n != s->n) return fail(COG_ERR_INVALID, "action_mask length != num_envs");
  DeviceGuard g(s->device);
  int rc = sampler_run(s, static_cast<const uint8_t *>(d_masks), s->stream, true);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(s->stream));
  return COG_OK;
}

int cog_sampler_sample(cog_sampler *s, const cog_action_mask_t *masks, size_t n) {
  if (!s || (!masks && n)) return fail(COG_ERR_INVALID, "NULL argument");
  if (n != s->n) return fail(COG_ERR_INVALID, "action_mask length != num_envs");
  DeviceGuard g(s->device);
  if (n) HIPCHK(hipMemcpyAsync(s->d_masks, masks, n * COG_MASK_BYTES, hipMemcpyHostToDevice, s->stream));
  return cog_sampler_sample_device(s, s->d_masks, n);
}

cog_action_t *cog_sampler_actions(cog_sampler *s) { return s ? s->h_actions : nullptr; }
void *cog_sampler_device_actions(cog_sampler *s) { return s ? (void *)s->d_actions : nullptr; }

// ---- runner ------------------------------------------------------------------------------
int cog_runner_create(cog_env *env, cog_sampler *s, size_t n_threads, uint32_t flags, cog_runner **out) {
  if (!env || !s || !out) return fail(COG_ERR_INVALID, "NULL argument");
  if (env->s.n != s->n) return fail(COG_ERR_INVALID, "env and sampler batch sizes differ");
  if (env->device != s->device) return fail(COG_ERR_INVALID, "env and sampler are on different devices");
  cog_runner *r = new cog_runner();
  r->env = env;
  r->smp = s;
  r->n_threads = n_threads;
  r->flags = flags;
  const char *cv = std::getenv("COG_RUNNER_CHUNK");        // default rollout steps per launch
  r->chunk = cv ? std::max(1, std::atoi(cv)) : 1;
  *out = r;
  return COG_OK;
}

void cog_runner_destroy(cog_runner *r) {
  if (!r) return;
  DeviceGuard g(r->env->device);
  (void)hipStreamSynchronize(r->env->stream);
  for (hipEvent_t ev : r->ev) (void)hipEventDestroy(ev);
  delete r;
}

size_t cog_runner_n_threads(const cog_runner *r) { return r ? r->n_threads : 0; }

static int runner_flush_sample(cog_runner *r) {
  if (!r->pending_sample) return COG_OK;
  r->pending_sample = false;
  // a lone sample reads the selected masks, as the reference runner's does (runner.h:26,48);
  // stored-mask sampling exists only fused with a step
  return sampler_run(r->smp, r->env->s.sel, r->env->stream, false);
}

static int runner_timing_event(cog_runner *r, hipEvent_t *out) {
  if (r->ev_used + 1 > r->ev.size()) {
    hipEvent_t ev;
    HIPCHK(hipEventCreate(&ev));
    r->ev.push_back(ev);
  }
  *out = r->ev[r->ev_used++];
  HIPCHK(hipEventRecord(*out, r->env->stream));
  return COG_OK;
}

// `steps` back-to-back fused sample+step launches; with timing on, one event pair brackets the
// batch (device time per launch = pair time / steps, the same quantity rocprofv3's kernel
// trace averages, without per-launch event overhead)
static int runner_launch_fused(cog_runner *r, int steps) {
  hipEvent_t ev;
  int rc;
  if (r->timing && (rc = runner_timing_event(r, &ev))) return rc;
  const int src = (r->flags & COG_RUNNER_STORED_MASKS) ? cog::MASK_STORED : cog::MASK_SELECTED;
  if (r->chunk > 1) {                                      // persistent kernels, chunk steps each
    for (int t = 0; t < steps; t += r->chunk)
      if (cog::launch_rollout(r->env->s, src, std::min(r->chunk, steps - t), r->smp->d_rng, r->smp->d_actions,
                              r->env->stream))
        return fail(COG_ERR_HIP, std::string("rollout launch failed: ") + hipGetErrorString(hipGetLastError()));
  } else {
    for (int t = 0; t < steps; t++)
      if (cog::launch_sample_step(r->env->s, src, r->smp->d_rng, r->smp->d_actions, r->env->stream))
        return fail(COG_ERR_HIP, std::string("sample_step launch failed: ") + hipGetErrorString(hipGetLastError()));
  }
  if (r->timing) {
    if ((rc = runner_timing_event(r, &ev))) return rc;
    r->timed_launches += (uint64_t)steps;
  }
  return COG_OK;
}

int cog_runner_sample(cog_runner *r) {
  if (!r) return fail(COG_ERR_INVALID, "runner is NULL");
  DeviceGuard g(r->env->device);
  int rc = runner_flush_sample(r);   // two samples in a row: the first one still runs
  if (rc) return rc;
  r->pending_sample = true;
  return COG_OK;
}

int cog_runner_step(cog_runner *r) {
  if (!r) return fail(COG_ERR_INVALID, "runner is NULL");
  DeviceGuard g(r->env->device);
  if (r->pending_sample) {
    r->pending_sample = false;
    return runner_launch_fused(r, 1);
  }
  if (cog::launch_step(r->env->s, r->smp->d_actions, r->env->stream))
    return fail(COG_ERR_HIP, std::string("step launch failed: ") + hipGetErrorString(hipGetLastError()));
  return COG_OK;
}

int cog_runner_rollout(cog_runner *r, int steps) {
  if (!r || steps < 0) return fail(COG_ERR_INVALID, "bad argument");
  DeviceGuard g(r->env->device);
  int rc = runner_flush_sample(r);
  if (rc) return rc;
  return steps ? runner_launch_fused(r, steps) : COG_OK;
}

int cog_runner_sync(cog_runner *r) {
  if (!r) return fail(COG_ERR_INVALID, "runner is NULL");
  DeviceGuard g(r->env->device);
  int rc = runner_flush_sample(r);
  if (rc) return rc;
  const bool host = !(r->flags & COG_RUNNER_DEVICE_VIEWS);
  if (host && r->smp->n)
    HIPCHK(hipMemcpyAsync(r->smp->h_actions, r->smp->d_actions, r->smp->n * COG_ACTION_BYTES,
                          hipMemcpyDeviceToHost, r->env->stream));
  return finish_steps(r->env, host);
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

int cog_runner_kernel_time(cog_runner *r, double *total_ms, uint64_t *launches) {
  if (!r) return fail(COG_ERR_INVALID, "runner is NULL");
  DeviceGuard g(r->env->device);
  HIPCHK(hipStreamSynchronize(r->env->stream));
  double acc = 0.0;
  for (size_t k = 0; k + 1 < r->ev_used; k += 2) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, r->ev[k], r->ev[k + 1]));
    acc += ms;
  }
  if (total_ms) *total_ms = acc;
  if (launches) *launches = r->timed_launches;
  r->ev_used = 0;
  r->timed_launches = 0;
  return COG_OK;
}

}  // extern "C"
