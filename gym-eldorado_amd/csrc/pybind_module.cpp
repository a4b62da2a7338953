// pybind_module.cpp -- `city_of_gold._city_of_gold`: the host C++ mirror of the reference's
// pybind11 surface (reference src/pybind/common.cpp, include/pybind/vectorized.h) on top of the
// C ABI of libcog_hip.so (include/cog.h).  It owns no game logic: every call forwards to the HIP
// engine, which fails loudly when no gfx950 device is present.
//
// numpy dtypes are registered from structs with the reference's field names, types and offsets
// (reference common.cpp:8-20, api.h:67-161) so structured views are drop-in compatible.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <array>
#include <cstdint>
#include <cstdlib>
#include <optional>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>
#include <algorithm>

#include "../../include/cog.h"

namespace py = pybind11;
using namespace pybind11::literals;

// ---- numpy record mirrors (bool fields typed bool so the dtype says '?') -------------------
struct DeckObs {
  std::array<uint8_t, 21> draw, hand, active, played, discard;
};
struct alignas(64) ActionMask {
  std::array<bool, 22> play;
  std::array<bool, 22> play_special;
  std::array<bool, 22> remove;
  std::array<bool, 7> move;
  std::array<bool, 19> get_from_shop;
};
struct SharedObservation {
  std::array<std::array<std::array<uint8_t, 7>, 48>, 48> map;
  uint8_t phase;
  std::array<float, 3> current_resources;
  std::array<uint8_t, 18> shop;
};
struct PlayerData {
  DeckObs obs;
  ActionMask action_mask;
};
struct alignas(64) ObsData {
  SharedObservation shared;
  std::array<PlayerData, 4> player_data;
};
struct alignas(64) ActionData {
  uint8_t play, play_special, remove, move, get_from_shop;
};
struct AgentInfo {
  uint8_t steps_taken;
  float returns;
  uint32_t travelled_hexes;
  uint8_t cards_added, cards_removed;
  uint32_t n_machete_uses, n_paddle_uses, n_coin_uses, n_card_uses;
};
struct alignas(64) Info {
  uint32_t total_length;
  std::array<AgentInfo, 4> agent_infos;
};
static_assert(sizeof(ObsData) == sizeof(cog_obs_t) && offsetof(ObsData, player_data) == COG_OBS_PLAYER0, "ObsData");
static_assert(offsetof(SharedObservation, current_resources) == COG_OBS_RES && offsetof(SharedObservation, shop) == COG_OBS_SHOP, "shared");
static_assert(sizeof(ActionMask) == sizeof(cog_action_mask_t) && offsetof(ActionMask, get_from_shop) == COG_MASK_SHOP, "mask");
static_assert(offsetof(PlayerData, action_mask) == COG_PD_MASK, "PlayerData");
static_assert(sizeof(ActionData) == sizeof(cog_action_t), "ActionData");
static_assert(sizeof(Info) == sizeof(cog_info_t) && offsetof(AgentInfo, n_machete_uses) == 16, "Info");

enum class Difficulty { EASY = 0, MEDIUM = 1, HARD = 2 };

static void check(int rc) {
  if (rc == COG_OK) return;
  std::string msg = cog_last_error();
  if (rc == COG_ERR_INVALID) throw py::value_error(msg);
  throw std::runtime_error(msg);
}

// Devices of a new handle (reference: one object owns every env, vectorized.h:185-214).
//   device=None: COG_DEVICES ("0,2,...": opt-in sharding over several GPUs), else COG_DEVICE
//                (pins the GPU, e.g. several ranks on one GPU), else LOCAL_RANK (one process per
//                GPU under torchrun), else GPU 0.  A handle never spans GPUs unless asked to, so
//                device views (device_tensors, step_device, sampler.dlpack) keep one shard.
//   device=int:  that GPU;  device=[d0, d1, ...]: one contiguous shard per entry.
static std::vector<int> parse_list(const char *v) {
  std::vector<int> out;
  const char *p = v;
  while (*p) {
    char *end = nullptr;
    const long d = std::strtol(p, &end, 10);
    if (end == p) throw py::value_error(std::string("bad device list: ") + v);
    out.push_back((int)d);
    p = *end == ',' ? end + 1 : end;
    if (*end && *end != ',') throw py::value_error(std::string("bad device list: ") + v);
  }
  if (out.empty()) throw py::value_error("empty device list");
  return out;
}
static std::vector<int> default_devices() {
  const char *v = std::getenv("COG_DEVICES");
  if (v && *v) return parse_list(v);
  const char *d = std::getenv("COG_DEVICE");
  if (d && *d) return {std::atoi(d)};
  const char *lr = std::getenv("LOCAL_RANK");
  if (lr && *lr) return {std::atoi(lr)};
  return {0};
}
static std::vector<int> devices_of(const py::object &device, size_t) {
  if (device.is_none()) return default_devices();
  if (py::isinstance<py::int_>(device)) return {device.cast<int>()};
  std::vector<int> out = device.cast<std::vector<int>>();
  if (out.empty()) throw py::value_error("device list is empty");
  return out;
}

// The env's outputs are read-only views (writeable=False): the reference's views alias the live
// engine state (common.h:98-101), so a write there changes the game; here the records live in HBM
// and the pinned views are the engine's copies, which it never reads back -- a write would be
// silently lost, so numpy refuses it instead ("assignment destination is read-only").  Inputs the
// caller fills (the sampler's actions, passed to env.step) stay writable.
static py::array readonly(py::array a) {
  a.attr("setflags")("write"_a = false);
  return a;
}
template <class T>
static py::array view(T *ptr, size_t n, py::handle base, bool writeable = false) {
  py::array a = py::array_t<T>({(py::ssize_t)n}, {(py::ssize_t)sizeof(T)}, ptr, base);
  return writeable ? a : readonly(a);
}

template <class T>
static const T *checked_records(const py::array &a, size_t n, const char *what) {
  const size_t item = sizeof(T);
  if (a.ndim() != 1 || (size_t)a.shape(0) != n)
    throw py::value_error(std::string(what) + ": expected a 1-D array of " + std::to_string(n) + " records");
  if ((size_t)a.itemsize() != item)
    throw py::value_error(std::string(what) + ": record size " + std::to_string(a.itemsize()) + " != " + std::to_string(item));
  if (!(a.flags() & py::array::c_style)) throw py::value_error(std::string(what) + ": array must be C-contiguous");
  return static_cast<const T *>(a.data());
}

// ---- DLPack export of the device views (zero-copy device consumers) ------
// The DLPack v0.x C structs (dlpack.h ABI), declared here rather than pulled from a framework.
struct DLDevice {
  int32_t device_type, device_id;
};
struct DLDataType {
  uint8_t code, bits;
  uint16_t lanes;
};
struct DLTensor {
  void *data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t *shape, *strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void *manager_ctx;
  void (*deleter)(DLManagedTensor *self);
};
constexpr int32_t kDLROCM = 10;
constexpr uint8_t kDLUInt = 1, kDLFloat = 2;

struct DLHolder {                     // owns the shape array and a reference to the owning object
  DLManagedTensor t;
  int64_t shape[2];
  PyObject *owner;
};
static void dl_delete(DLManagedTensor *self) {
  DLHolder *h = reinterpret_cast<DLHolder *>(self->manager_ctx);
  {
    py::gil_scoped_acquire g;
    Py_XDECREF(h->owner);
  }
  delete h;
}
// a "dltensor" capsule over n records of `width` elements of (code, bits) at device address p
// (width 0: a 1-D tensor of n elements); the consumer's tensor keeps `owner` alive
static py::capsule dl_capsule(void *p, int device, size_t n, int64_t width, uint8_t code, uint8_t bits, py::handle owner) {
  DLHolder *h = new DLHolder();
  h->shape[0] = (int64_t)n;
  h->shape[1] = width;
  h->owner = owner.ptr();
  Py_XINCREF(h->owner);
  DLTensor &t = h->t.dl_tensor;
  t.data = p;
  t.device = DLDevice{kDLROCM, device};
  t.ndim = width > 0 ? 2 : 1;
  t.dtype = DLDataType{code, bits, 1};
  t.shape = h->shape;
  t.strides = nullptr;                // compact row-major
  t.byte_offset = 0;
  h->t.manager_ctx = h;
  h->t.deleter = dl_delete;
  return py::capsule(&h->t, "dltensor", [](PyObject *cap) {
    // only an unconsumed capsule still owns its tensor (consumers rename it "used_dltensor")
    if (PyCapsule_IsValid(cap, "dltensor")) {
      auto *m = static_cast<DLManagedTensor *>(PyCapsule_GetPointer(cap, "dltensor"));
      if (m && m->deleter) m->deleter(m);
    }
  });
}

// ---- vec env (py_vec_env, vectorized.h:25-105) -------------------------------------------
class VecEnv {
 public:
  VecEnv(size_t n, const py::object &device) : n_(n) {
    const std::vector<int> d = devices_of(device, n);
    check(cog_env_create_multi(n, d.data(), (int)d.size(), &h_));
  }
  ~VecEnv() { cog_env_destroy(h_); }
  VecEnv(const VecEnv &) = delete;
  VecEnv &operator=(const VecEnv &) = delete;

  void reset_default() { check(cog_env_reset_default(h_)); }
  void reset(uint32_t seed, uint8_t n_players, uint8_t n_pieces, Difficulty d, uint32_t max_steps, bool render) {
    check(cog_env_reset(h_, seed, n_players, n_pieces, (int32_t)d, max_steps, render));
  }
  void step(const py::array &actions) {
    const ActionData *a = checked_records<ActionData>(actions, n_, "actions");
    check(cog_env_step(h_, reinterpret_cast<const cog_action_t *>(a), n_));
  }
  cog_env_views views() {
    cog_env_views v;
    check(cog_env_get_views(h_, &v));
    return v;
  }
  cog_env_views shard_views(int k) {
    cog_env_views v;
    check(cog_env_shard_views(h_, k, &v));
    return v;
  }
  int num_shards() const {
    int k = 0;
    check(cog_env_num_shards(h_, &k));
    return k;
  }
  size_t num_envs() const { return n_; }
  cog_env *handle() { return h_; }

 private:
  size_t n_;
  cog_env *h_ = nullptr;
};

// ---- vec sampler (py_vec_action_sampler, vectorized.h:107-127) ----------------------------
class VecSampler {
 public:
  VecSampler(size_t n, std::optional<size_t> seed, const py::object &device, uint64_t first_index) : n_(n) {
    const uint32_t s = (uint32_t)seed.value_or(std::random_device{}());   // u32 as in vectorized.h:113
    const std::vector<int> d = devices_of(device, n);
    check(cog_sampler_create_at(n, s, first_index, d.data(), (int)d.size(), &h_));
  }
  ~VecSampler() { cog_sampler_destroy(h_); }
  VecSampler(const VecSampler &) = delete;
  VecSampler &operator=(const VecSampler &) = delete;
  void sample(const py::array &masks) {
    const ActionMask *m = checked_records<ActionMask>(masks, n_, "action_mask");
    check(cog_sampler_sample(h_, reinterpret_cast<const cog_action_mask_t *>(m), n_));
  }
  ActionData *actions() { return reinterpret_cast<ActionData *>(cog_sampler_actions(h_)); }
  size_t num_envs() const { return n_; }
  cog_sampler *handle() { return h_; }

 private:
  size_t n_;
  cog_sampler *h_ = nullptr;
};

// ---- runner (py_threaded_runner, vectorized.h:129-161) ------------------------------------
class Runner {
 public:
  Runner(VecEnv &env, VecSampler &smp, std::optional<size_t> n_threads, bool device_views, bool stored_masks)
      : env_(env), smp_(smp) {
    uint32_t flags = (device_views ? COG_RUNNER_DEVICE_VIEWS : 0u) | (stored_masks ? COG_RUNNER_STORED_MASKS : 0u);
    check(cog_runner_create(env.handle(), smp.handle(), n_threads.value_or(std::thread::hardware_concurrency()), flags, &h_));
  }
  ~Runner() { cog_runner_destroy(h_); }
  Runner(const Runner &) = delete;
  Runner &operator=(const Runner &) = delete;
  size_t n_threads() const { return cog_runner_n_threads(h_); }
  void sample() { check(cog_runner_sample(h_)); }
  void step() { check(cog_runner_step(h_)); }
  void sync() { check(cog_runner_sync(h_)); }
  void step_sync() {
    check(cog_runner_step(h_));
    check(cog_runner_sync(h_));
  }
  void rollout(int steps) { check(cog_runner_rollout(h_, steps)); }
  void set_timing(bool on) { check(cog_runner_set_timing(h_, on)); }
  void set_chunk(int k) { check(cog_runner_set_chunk(h_, k)); }
  py::tuple kernel_time() {
    double ms = 0;
    uint64_t k = 0;
    check(cog_runner_kernel_time(h_, &ms, &k));
    return py::make_tuple(ms, k);
  }
  VecEnv &env() { return env_; }
  VecSampler &sampler() { return smp_; }

 private:
  VecEnv &env_;
  VecSampler &smp_;
  cog_runner *h_ = nullptr;
};

PYBIND11_MODULE(_city_of_gold, m) {
  m.doc() = "MI355X-native City of Gold engine: host bindings over libcog_hip.so";
  PYBIND11_NUMPY_DTYPE(DeckObs, draw, hand, active, played, discard);
  PYBIND11_NUMPY_DTYPE(ActionMask, play, play_special, remove, get_from_shop, move);
  PYBIND11_NUMPY_DTYPE(PlayerData, obs, action_mask);
  PYBIND11_NUMPY_DTYPE(SharedObservation, map, phase, shop, current_resources);
  PYBIND11_NUMPY_DTYPE(ObsData, shared, player_data);
  PYBIND11_NUMPY_DTYPE(ActionData, play, play_special, remove, move, get_from_shop);
  PYBIND11_NUMPY_DTYPE(AgentInfo, steps_taken, returns, travelled_hexes, cards_added, cards_removed,
                       n_machete_uses, n_paddle_uses, n_coin_uses, n_card_uses);
  PYBIND11_NUMPY_DTYPE(Info, total_length, agent_infos);

  py::enum_<Difficulty>(m, "Difficulty")
      .value("EASY", Difficulty::EASY)
      .value("MEDIUM", Difficulty::MEDIUM)
      .value("HARD", Difficulty::HARD)
      .export_values();

  m.attr("ObsData") = py::dtype::of<ObsData>();
  m.attr("ActionMask") = py::dtype::of<ActionMask>();
  m.attr("ActionData") = py::dtype::of<ActionData>();
  m.attr("Info") = py::dtype::of<Info>();
  m.attr("DeckObs") = py::dtype::of<DeckObs>();
  m.attr("ABI_VERSION") = cog_abi_version();
  m.def("device_count", []() {
    int n = 0;
    check(cog_device_count(&n));
    return n;
  });
  m.def(
      "rollout_kind",
      [](size_t n, int n_players, bool stored_masks) {
        static const char *names[] = {"duo", "wave", "pipe", "trio"};
        const int k = cog_rollout_kind(n, n_players, stored_masks ? 1 : 0);
        return std::string(k >= 0 && k < 4 ? names[k] : "?");
      },
      "n"_a, "n_players"_a = 4, "stored_masks"_a = false,
      "the persistent rollout kernel launched for a shard of n envs: duo | pipe | wave | trio");
  m.def("default_devices", []() { return default_devices(); },
        "the GPUs a handle created with device=None uses (COG_DEVICES, else COG_DEVICE, else LOCAL_RANK, else 0)");
  m.def(
      "time_copy",
      [](int device, size_t bytes, int iters) {
        double gbs = 0.0;
        check(cog_time_copy(device, bytes, iters, &gbs));
        return gbs;
      },
      "device"_a = 0, "bytes"_a = (size_t)1 << 31, "iters"_a = 5,
      "read + write GB/s of the engine's device copy kernel (measurement)");
  m.def(
      "time_stream_mix",
      [](int device, size_t bytes, int iters) {
        double gbs = 0.0;
        check(cog_time_stream_mix(device, bytes, iters, &gbs));
        return gbs;
      },
      "device"_a = 0, "bytes"_a = (size_t)1 << 28, "iters"_a = 5,
      "read + write GB/s of a stream with the encode's 1:7 read:write mix (measurement)");

  py::class_<VecEnv>(m, "VecEnvBase", py::dynamic_attr())
      .def(py::init<size_t, const py::object &>(), "n_envs"_a, "device"_a = py::none())
      .def("reset", &VecEnv::reset_default, "Reset all environments, keeping parameters (vectorized.h:187-195)")
      .def("reset", &VecEnv::reset, "seed"_a, "n_players"_a, "n_pieces"_a, "difficulty"_a, "max_steps"_a, "render"_a)
      .def("step", &VecEnv::step, "actions"_a)
      .def_property_readonly("num_envs", &VecEnv::num_envs)
      .def_property_readonly("observations", [](py::object self) {
        VecEnv &e = self.cast<VecEnv &>();
        auto v = e.views();
        return view(reinterpret_cast<ObsData *>(v.observations), v.n_envs, self);
      })
      .def_property_readonly("selected_action_masks", [](py::object self) {
        VecEnv &e = self.cast<VecEnv &>();
        auto v = e.views();
        return view(reinterpret_cast<ActionMask *>(v.selected_action_masks), v.n_envs, self);
      })
      .def_property_readonly("agent_selection", [](py::object self) {
        VecEnv &e = self.cast<VecEnv &>();
        auto v = e.views();
        return view(v.agent_selection, v.n_envs, self);
      })
      .def_property_readonly("dones", [](py::object self) {
        VecEnv &e = self.cast<VecEnv &>();
        auto v = e.views();
        return view(reinterpret_cast<bool *>(v.dones), v.n_envs, self);
      })
      .def_property_readonly("rewards", [](py::object self) {
        VecEnv &e = self.cast<VecEnv &>();
        auto v = e.views();
        return readonly(py::array_t<float>({(py::ssize_t)v.n_envs, (py::ssize_t)4}, {(py::ssize_t)16, (py::ssize_t)4},
                                           v.rewards, self));
      })
      .def_property_readonly("infos", [](py::object self) {
        VecEnv &e = self.cast<VecEnv &>();
        auto v = e.views();
        return view(reinterpret_cast<Info *>(v.infos), v.n_envs, self);
      })
      .def_property_readonly("num_shards", &VecEnv::num_shards)
      .def("shard_info", [](VecEnv &e, int k) {
        size_t first = 0, count = 0;
        int dev = 0;
        check(cog_env_shard_info(e.handle(), k, &first, &count, &dev));
        return py::make_tuple(first, count, dev);
      }, "shard"_a)
      .def("device_pointers", [](VecEnv &e, int k) {
        auto v = e.shard_views(k);
        return py::dict("observations"_a = (uintptr_t)v.d_observations,
                        "selected_action_masks"_a = (uintptr_t)v.d_selected_action_masks,
                        "rewards"_a = (uintptr_t)v.d_rewards, "dones"_a = (uintptr_t)v.d_dones,
                        "agent_selection"_a = (uintptr_t)v.d_agent_selection, "infos"_a = (uintptr_t)v.d_infos);
      }, "shard"_a = 0)
      .def("dlpack", [](py::object self, const std::string &name, int k) {
        // one device view of shard k as a DLPack capsule (torch.from_dlpack, TensorDict); rows are records
        VecEnv &e = self.cast<VecEnv &>();
        auto v = e.shard_views(k);
        size_t first = 0, count = 0;
        int dev = 0;
        check(cog_env_shard_info(e.handle(), k, &first, &count, &dev));
        const size_t n = v.n_envs;
        if (name == "observations") return dl_capsule(v.d_observations, dev, n, sizeof(ObsData), kDLUInt, 8, self);
        if (name == "selected_action_masks")
          return dl_capsule(v.d_selected_action_masks, dev, n, sizeof(ActionMask), kDLUInt, 8, self);
        if (name == "rewards") return dl_capsule(v.d_rewards, dev, n, 4, kDLFloat, 32, self);
        if (name == "dones") return dl_capsule(v.d_dones, dev, n, 0, kDLUInt, 8, self);
        if (name == "agent_selection") return dl_capsule(v.d_agent_selection, dev, n, 0, kDLUInt, 8, self);
        if (name == "infos") return dl_capsule(v.d_infos, dev, n, sizeof(Info), kDLUInt, 8, self);
        throw py::value_error("no device view named " + name);
      }, "name"_a, "shard"_a = 0)
      .def("step_device", [](VecEnv &e, uintptr_t d_actions, int64_t stream) {
        // step with ActionData records already in device memory (e.g. a torch tensor's data_ptr()),
        // ordered after the work queued on `stream` (a hipStream_t handle, 0 = the null stream;
        // -1: no ordering)
        check(cog_env_step_device_stream(e.handle(), reinterpret_cast<const void *>(d_actions), e.num_envs(),
                                         stream < 0 ? COG_NO_STREAM : reinterpret_cast<void *>((uintptr_t)stream)));
      }, "d_actions"_a, "stream"_a = -1)
      .def("wait_stream", [](VecEnv &e, uintptr_t stream, int k) {
        check(cog_env_wait_stream(e.handle(), k, reinterpret_cast<void *>(stream)));
      }, "stream"_a, "shard"_a = 0)
      .def("signal_stream", [](VecEnv &e, uintptr_t stream, int k) {
        check(cog_env_signal_stream(e.handle(), k, reinterpret_cast<void *>(stream)));
      }, "stream"_a, "shard"_a = 0)
      .def("invalidate_device", [](VecEnv &e, int64_t stream) {
        // the caller wrote device records: rebuild the engine's mirrors of them (cog.h), ordered
        // after the work queued on `stream` (-1: no ordering)
        check(cog_env_invalidate_device(e.handle(), stream < 0 ? COG_NO_STREAM : reinterpret_cast<void *>((uintptr_t)stream)));
      }, "stream"_a = -1)
      .def("set_autoreset", [](VecEnv &e, bool on) { check(cog_env_set_autoreset(e.handle(), on ? 1 : 0)); }, "on"_a)
      .def("stream", [](VecEnv &e, int k) { return (uintptr_t)cog_env_shard_stream(e.handle(), k); }, "shard"_a = 0)
      .def("hazards", [](VecEnv &e) {
        py::array_t<uint32_t> per((py::ssize_t)e.num_envs());
        uint32_t acc = 0;
        check(cog_env_hazards(e.handle(), &acc, per.mutable_data()));
        return py::make_tuple(acc, per);
      })
      .def("clear_hazards", [](VecEnv &e) { check(cog_env_clear_hazards(e.handle())); })
      .def("sync_host", [](VecEnv &e) { check(cog_env_sync_host(e.handle())); })
      .def("time_encode", [](VecEnv &e, int iters, int variant) {
        double ms = 0;
        check(cog_env_time_encode(e.handle(), iters, variant, &ms));
        return ms;
      }, "iters"_a = 20, "variant"_a = 0);

  py::class_<VecSampler>(m, "VecSamplerBase", py::dynamic_attr())
      .def(py::init<size_t, std::optional<size_t>, const py::object &, uint64_t>(), "n_envs"_a, "seed"_a = py::none(),
           "device"_a = py::none(), "first_index"_a = 0)
      .def("get_actions", [](py::object self) {
        VecSampler &s = self.cast<VecSampler &>();
        return view(s.actions(), s.num_envs(), self, true);   // an input of env.step: writable
      })
      .def("sample", &VecSampler::sample, "action_mask"_a)
      .def("spec_stats", [](VecSampler &s) {
        uint64_t samples = 0, hits = 0;
        check(cog_sampler_spec_stats(s.handle(), &samples, &hits));
        return py::make_tuple(samples, hits);
      }, "(samples, speculative samples taken): cog_sampler_spec_stats")
      .def("device_actions", [](VecSampler &s, int k) {
        return (uintptr_t)cog_sampler_shard_device_actions(s.handle(), k);
      }, "shard"_a = 0)
      .def_property_readonly("num_shards", [](VecSampler &s) {
        int k = 0;
        check(cog_sampler_num_shards(s.handle(), &k));
        return k;
      })
      .def("dlpack", [](py::object self) {       // the device actions (ActionData rows), single shard
        VecSampler &s = self.cast<VecSampler &>();
        int k = 0;
        check(cog_sampler_num_shards(s.handle(), &k));
        if (k != 1) throw py::value_error("dlpack() of a multi-shard sampler: use device_actions(shard)");
        return dl_capsule(cog_sampler_device_actions(s.handle()), cog_sampler_device(s.handle()), s.num_envs(),
                          sizeof(ActionData), kDLUInt, 8, self);
      });

  py::class_<Runner>(m, "RunnerBase", py::dynamic_attr())
      .def(py::init<VecEnv &, VecSampler &, std::optional<size_t>, bool, bool>(), "env"_a, "sampler"_a,
           "n_threads"_a = py::none(), "device_views"_a = false, "stored_masks"_a = false,
           py::keep_alive<1, 2>(), py::keep_alive<1, 3>())
      .def("get_envs", &Runner::env, py::return_value_policy::reference_internal)
      .def("get_samplers", &Runner::sampler, py::return_value_policy::reference_internal)
      .def("get_n_threads", &Runner::n_threads)
      .def("get_actions", [](py::object self) {
        Runner &r = self.cast<Runner &>();
        return view(r.sampler().actions(), r.sampler().num_envs(), self);
      })
      .def("get_action_masks", [](py::object self) {
        Runner &r = self.cast<Runner &>();
        auto v = r.env().views();
        return view(reinterpret_cast<ActionMask *>(v.selected_action_masks), v.n_envs, self);
      })
      .def("sample", &Runner::sample)
      .def("step", &Runner::step)
      .def("step_sync", &Runner::step_sync)
      .def("sync", &Runner::sync)
      .def("rollout", &Runner::rollout, "steps"_a)
      .def("set_timing", &Runner::set_timing, "enable"_a)
      .def("set_chunk", &Runner::set_chunk, "steps_per_launch"_a)
      .def("kernel_time", &Runner::kernel_time);
}
