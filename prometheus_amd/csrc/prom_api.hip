// C-ABI layer of libprom_hip.so (declared in include/prom_hip.h).  Host code only: argument checks,
// device memory owned by the context, H2D/D2H copies and kernel launches on the context's stream.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <exception>
#include <map>
#include <mutex>
#include <thread>

#include "prom_internal.h"

using prom::DevBuf;
using prom::Error;

namespace {

template <class F>
int32_t guarded(prom_ctx* ctx, F&& f) {
  if (!ctx) return PROM_E_ARG;
  try {
    PROM_HIP(hipSetDevice(ctx->device));
    f();
    ctx->err.clear();
    return PROM_OK;
  } catch (const Error& e) {
    ctx->err = e.what();
    return e.code;
  } catch (const std::exception& e) {
    ctx->err = e.what();
    return PROM_E_HIP;
  }
}

template <class T>
void upload(DevBuf& b, const T* h, int64_t n, hipStream_t s) {
  b.ensure(sizeof(T) * (size_t)std::max<int64_t>(n, 1));
  if (n > 0) PROM_HIP(hipMemcpyAsync(b.p, h, sizeof(T) * (size_t)n, hipMemcpyHostToDevice, s));
}

template <class T>
void download(T* h, const DevBuf& b, int64_t n, hipStream_t s) {
  if (n > 0) PROM_HIP(hipMemcpyAsync(h, b.p, sizeof(T) * (size_t)n, hipMemcpyDeviceToHost, s));
}

prom::DensityDev to_dev(const prom_density_model& m) {
  prom::DensityDev d{};
  d.kind = m.kind;
  for (int i = 0; i < 8; ++i) d.p[i] = m.p[i];
  // power law with a small integral exponent q (the setup files' q_esc, e.g. 6): (R / r)^q by repeated
  // squaring on the device (pad = q + 1) instead of a general pow.  Each squaring doubles the relative error
  // already carried, so the error grows about linearly in q: q <= 8 keeps it within ~8 ulp of pow
  // (test_density_plugins, q = 6); larger exponents take pow
  if (m.kind == PROM_DENSITY_POWERLAW && m.p[2] >= 0.0 && m.p[2] <= 8.0 && m.p[2] == std::floor(m.p[2]))
    d.pad = (int32_t)m.p[2] + 1;
  return d;
}

bool valid_kind(int32_t k) { return k >= PROM_DENSITY_BAROMETRIC && k <= PROM_DENSITY_GRIDDED; }

// GRIDDED: grid sizes from p[0..2] (each >= 2) and the packed length of [gx, gy, gz, values]
bool gridded_dims(const prom_density_model& m, int64_t* nx, int64_t* ny, int64_t* nz, int64_t* len) {
  for (int i = 0; i < 3; ++i)
    if (!(m.p[i] >= 2.0 && m.p[i] <= 1.0e6 && m.p[i] == std::floor(m.p[i]))) return false;
  *nx = (int64_t)m.p[0];
  *ny = (int64_t)m.p[1];
  *nz = (int64_t)m.p[2];
  *len = *nx + *ny + *nz + *nx * *ny * *nz;
  return *nx * *ny * *nz < ((int64_t)1 << 31);
}

// Table slots: an upload takes the lowest free slot (freed ids are reused), so a loop that builds and
// drops tables keeps the context's device memory flat.
template <class T>
int32_t store_table(std::vector<T>& v, T&& t) {
  t.live = true;
  for (size_t i = 0; i < v.size(); ++i)
    if (!v[i].live) {
      v[i] = std::move(t);
      return (int32_t)i;
    }
  v.push_back(std::move(t));
  return (int32_t)v.size() - 1;
}

template <class T>
bool table_ok(const std::vector<T>& v, int32_t id) {
  return id >= 0 && id < (int32_t)v.size() && v[id].live;
}

// Pinned host pool behind prom_host_alloc / prom_host_free: buffers keyed by address, each either in use
// or cached for reuse; the total (in use + cached) stays under the cap, idle buffers are released first
struct PinnedPool {
  struct Buf {
    size_t cap;
    bool used;
  };
  std::mutex mu;
  std::map<char*, Buf> bufs;
  size_t total = 0;
  size_t cap_bytes() const {
    const char* e = std::getenv("PROM_PINNED_CAP_MB");
    const long long mb = e ? std::atoll(e) : 4096;
    return (size_t)std::max(0LL, mb) << 20;
  }
  // in-use buffer holding [p, p + n)
  bool holds(const void* p, size_t n) {
    std::lock_guard<std::mutex> g(mu);
    const char* c = static_cast<const char*>(p);
    auto it = bufs.upper_bound(const_cast<char*>(c));
    if (it == bufs.begin()) return false;
    --it;
    return it->second.used && c >= it->first && c + n <= it->first + it->second.cap;
  }
};

PinnedPool& pinned_pool() {
  static PinnedPool* pool = new PinnedPool();   // never destroyed: buffers may outlive static teardown
  return *pool;
}

// prom_transit_set's inputs: small arrays are appended to a host image at add() (the callers' temporaries
// may die before the flush) and reach the device as one DMA of [descriptors | data] plus one scatter kernel,
// instead of a pageable copy each; large arrays are copied directly (one DMA when they sit in the pinned
// pool, e.g. the wavelength grid of a Transit)
struct Stager {
  static constexpr size_t kSmall = (size_t)256 << 10;
  std::vector<char> img;
  std::vector<std::pair<DevBuf*, int64_t>> ent;   // destination, offset in img
  std::vector<int64_t> len;
  template <class T>
  void add(DevBuf& b, const T* h, int64_t n, hipStream_t s) {
    b.ensure(sizeof(T) * (size_t)std::max<int64_t>(n, 1));
    if (n <= 0) return;
    const size_t bytes = sizeof(T) * (size_t)n;
    if (bytes > kSmall) {
      PROM_HIP(hipMemcpyAsync(b.p, h, bytes, hipMemcpyHostToDevice, s));
      return;
    }
    const size_t off = (img.size() + 15) & ~(size_t)15;
    img.resize(off + bytes);
    std::memcpy(img.data() + off, h, bytes);
    ent.push_back({&b, (int64_t)off});
    len.push_back((int64_t)bytes);
  }
  void flush(prom_ctx* ctx, hipStream_t s) {
    if (ent.empty()) return;
    const size_t n = ent.size();
    const size_t head = (sizeof(prom::ScatterDesc) * n + 255) & ~(size_t)255;
    const size_t total = head + img.size();
    if (ctx->upin_cap < total) {
      // nothing reads the old staging: every set ends with a stream synchronisation
      if (ctx->upin) PROM_HIP(hipHostFree(ctx->upin));
      ctx->upin = nullptr;
      ctx->upin_cap = 0;
      const size_t cap = std::max<size_t>(total * 2, (size_t)1 << 20);
      PROM_HIP(hipHostMalloc(&ctx->upin, cap, hipHostMallocDefault));
      ctx->upin_cap = cap;
    }
    ctx->ustage.ensure(ctx->upin_cap);
    char* dbase = static_cast<char*>(ctx->ustage.p);
    auto* d = static_cast<prom::ScatterDesc*>(ctx->upin);
    for (size_t i = 0; i < n; ++i) d[i] = prom::ScatterDesc{ent[i].first->p, (int64_t)head + ent[i].second, len[i]};
    std::memcpy(static_cast<char*>(ctx->upin) + head, img.data(), img.size());
    PROM_HIP(hipMemcpyAsync(dbase, ctx->upin, total, hipMemcpyHostToDevice, s));
    prom::launch_scatter(s, dbase, reinterpret_cast<const prom::ScatterDesc*>(dbase), (int32_t)n);
    img.clear();
    ent.clear();
    len.clear();
  }
};

}  // namespace

extern "C" {

int32_t prom_host_alloc(int64_t bytes, void** out) {
  if (!out || bytes < 0) return PROM_E_ARG;
  *out = nullptr;
  PinnedPool& pp = pinned_pool();
  const size_t want = std::max<size_t>(((size_t)bytes + ((size_t)1 << 21) - 1) & ~(((size_t)1 << 21) - 1),
                                       (size_t)1 << 21);
  std::lock_guard<std::mutex> g(pp.mu);
  char* best = nullptr;
  for (auto& kv : pp.bufs)
    if (!kv.second.used && kv.second.cap >= want && kv.second.cap <= 2 * want &&
        (!best || kv.second.cap < pp.bufs[best].cap))
      best = kv.first;
  if (best) {
    pp.bufs[best].used = true;
    *out = best;
    return PROM_OK;
  }
  const size_t cap = pp.cap_bytes();
  for (auto it = pp.bufs.begin(); pp.total + want > cap && it != pp.bufs.end();) {
    if (!it->second.used) {
      (void)hipHostFree(it->first);
      pp.total -= it->second.cap;
      it = pp.bufs.erase(it);
    } else {
      ++it;
    }
  }
  if (pp.total + want > cap) return PROM_E_NOMEM;
  void* p = nullptr;
  if (hipHostMalloc(&p, want, hipHostMallocPortable) != hipSuccess || !p) return PROM_E_NOMEM;
  pp.bufs[static_cast<char*>(p)] = PinnedPool::Buf{want, true};
  pp.total += want;
  *out = p;
  return PROM_OK;
}

int32_t prom_host_free(void* p) {
  PinnedPool& pp = pinned_pool();
  std::lock_guard<std::mutex> g(pp.mu);
  auto it = pp.bufs.find(static_cast<char*>(p));
  if (!p || it == pp.bufs.end() || !it->second.used) return PROM_E_ARG;
  it->second.used = false;
  return PROM_OK;
}

int32_t prom_abi_version(void) { return PROM_ABI_VERSION; }

int32_t prom_device_count(int32_t* count) {
  if (!count) return PROM_E_ARG;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return PROM_OK;
}

int32_t prom_create(int32_t device, prom_ctx** out) {
  if (!out) return PROM_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return PROM_E_HIP;
  prom_ctx* ctx = new (std::nothrow) prom_ctx();
  if (!ctx) return PROM_E_NOMEM;
  ctx->device = device;
  bool ok = hipSetDevice(device) == hipSuccess;
  for (int i = 0; ok && i < prom::kMaxSlots; ++i)
    ok = hipStreamCreateWithFlags(&ctx->streams[i], hipStreamNonBlocking) == hipSuccess;
  ctx->stream = ctx->streams[0];
  if (const char* e = std::getenv("PROM_PIPELINE")) ctx->pipeline = std::max(1, std::min(prom::kMaxSlots, std::atoi(e)));
  if (!ok) {
    delete ctx;
    return PROM_E_HIP;
  }
  for (int i = 0; i < prom::kMaxSlots; ++i) {
    if (hipEventCreateWithFlags(&ctx->fork_ev[i], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->join_ev[i], hipEventDisableTiming) != hipSuccess) {
      prom_destroy(ctx);
      return PROM_E_HIP;
    }
  }
  for (auto& e : ctx->ev) {
    if (hipEventCreate(&e) != hipSuccess) {
      delete ctx;
      return PROM_E_HIP;
    }
  }

  *out = ctx;
  return PROM_OK;
}

static void drop_graphs(prom::TransitDev& tr) {
  for (auto& g : tr.gexec)
    if (g) {
      (void)hipGraphExecDestroy(g);
      g = nullptr;
    }
}

void prom_destroy(prom_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (auto st : ctx->streams)
    if (st) (void)hipStreamSynchronize(st);
  drop_graphs(ctx->tr);
  for (auto& e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : ctx->tev) (void)hipEventDestroy(e);
  for (auto& e : ctx->pin_ev) (void)hipEventDestroy(e);
  for (int i = 0; i < prom::kMaxSlots; ++i) {
    if (ctx->fork_ev[i]) (void)hipEventDestroy(ctx->fork_ev[i]);
    if (ctx->join_ev[i]) (void)hipEventDestroy(ctx->join_ev[i]);
  }
  if (ctx->pin) (void)hipHostFree(ctx->pin);
  if (ctx->upin) (void)hipHostFree(ctx->upin);
  for (auto& st : ctx->streams)
    if (st) {
      (void)hipStreamSynchronize(st);
      (void)hipStreamDestroy(st);
    }
  delete ctx;  // DevBuf destructors free device memory
}

const char* prom_last_error(const prom_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int32_t prom_synchronize(prom_ctx* ctx) {
  return guarded(ctx, [&] {
    for (auto st : ctx->streams) PROM_HIP(hipStreamSynchronize(st));
  });
}

// ------------------------------------------------------------------------------ tables
// Bucket directory of a table's nodes: n_dir = 4 n equal buckets over [x0, x[n-1]], dir[j] = number of
// nodes <= x0 + j h.  The tau kernel starts its np.interp bracket search from buckets j, j+1 of a
// target and verifies the bracket, so rounding in j only costs steps, never correctness.
static void build_directory(prom_ctx* ctx, prom::AtomTable& t, const double* x, int64_t n) {
  const int64_t nd = std::max<int64_t>(1, std::min<int64_t>(4 * n, (int64_t)1 << 26));
  const double x0 = x[0], span = x[n - 1] - x[0];
  std::vector<int32_t> d(nd + 1);
  const double h = span > 0.0 ? span / (double)nd : 1.0;
  for (int64_t j = 0; j <= nd; ++j) {
    const double b = x0 + (double)j * h;
    d[j] = (int32_t)(std::upper_bound(x, x + n, b) - x);
  }
  upload(t.dir, d.data(), nd + 1, ctx->stream);
  t.rec.ensure(sizeof(double4) * n);
  ctx->scratch[5].ensure(sizeof(double) * std::max<int64_t>(n, 1));
  ctx->scratch[4].ensure(sizeof(double) * 1024);
  prom::launch_table_recs(ctx->stream, t.x.as<double>(), t.y.as<double>(), n, t.rec.as<double4>(),
                          ctx->scratch[5].as<double>());
  t.amax = prom::reduce_max(ctx->stream, ctx->scratch[5].as<double>(), n, ctx->scratch[4].as<double>());
  t.hx.assign(x, x + n);
  t.n_dir = (int32_t)nd;
  t.dir_x0 = x0;
  t.dir_inv_h = span > 0.0 ? 1.0 / h : 0.0;
}

int32_t prom_table_upload(prom_ctx* ctx, int64_t n, const double* x, const double* log_sigma,
                          double offset, int32_t* table_id) {
  return guarded(ctx, [&] {
    PROM_REQUIRE(n >= 1 && x && log_sigma && table_id, "prom_table_upload: bad arguments");
    PROM_REQUIRE(n < ((int64_t)1 << 31), "prom_table_upload: more than 2^31 - 1 nodes");
    for (int64_t i = 1; i < n; ++i) PROM_REQUIRE(!(x[i] < x[i - 1]), "prom_table_upload: x must be non-decreasing");
    prom::AtomTable t;
    upload(t.x, x, n, ctx->stream);
    upload(t.y, log_sigma, n, ctx->stream);
    t.n = n;
    t.offset = offset;
    double m = -INFINITY;
    for (int64_t i = 0; i < n; ++i) m = std::max(m, log_sigma[i]);
    t.ymax = m;
    build_directory(ctx, t, x, n);
    PROM_HIP(hipStreamSynchronize(ctx->stream));
    t.gen = ++ctx->table_gen;
    *table_id = store_table(ctx->tables, std::move(t));
  });
}

static void voigt_common(prom_ctx* ctx, int64_t n, const double* x, int32_t n_lines, const double* lw,
                         const double* lg, const double* lc, DevBuf& dx) {
  PROM_REQUIRE(n >= 0 && (n == 0 || x) && n_lines >= 0 && (n_lines == 0 || (lw && lg && lc)),
               "voigt: bad arguments");
  upload(dx, x, n, ctx->stream);
  upload(ctx->scratch[1], lw, n_lines, ctx->stream);
  upload(ctx->scratch[2], lg, n_lines, ctx->stream);
  upload(ctx->scratch[3], lc, n_lines, ctx->stream);
}

int32_t prom_table_build_voigt(prom_ctx* ctx, int64_t n, const double* x, int32_t n_lines,
                               const double* line_wavelength, const double* line_gamma,
                               const double* line_coef, double sigma_v, double c_light,
                               double offset, int32_t* table_id, double* log_sigma_out) {
  return guarded(ctx, [&] {
    PROM_REQUIRE(n >= 1 && table_id, "prom_table_build_voigt: bad arguments");
    PROM_REQUIRE(n < ((int64_t)1 << 31), "prom_table_build_voigt: more than 2^31 - 1 nodes");
    for (int64_t i = 1; i < n; ++i) PROM_REQUIRE(!(x[i] < x[i - 1]), "prom_table_build_voigt: x must be non-decreasing");
    prom::AtomTable t;
    voigt_common(ctx, n, x, n_lines, line_wavelength, line_gamma, line_coef, t.x);
    t.y.ensure(sizeof(double) * n);
    prom::launch_voigt(ctx->stream, t.x.as<double>(), n, ctx->scratch[1].as<double>(),
                       ctx->scratch[2].as<double>(), ctx->scratch[3].as<double>(), n_lines, sigma_v, c_light,
                       offset, 1, t.y.as<double>());
    ctx->scratch[4].ensure(sizeof(double) * 1024);
    t.ymax = prom::reduce_max(ctx->stream, t.y.as<double>(), n, ctx->scratch[4].as<double>());
    t.n = n;
    t.offset = offset;
    build_directory(ctx, t, x, n);
    PROM_HIP(hipStreamSynchronize(ctx->stream));
    if (log_sigma_out) {
      download(log_sigma_out, t.y, n, ctx->stream);
      PROM_HIP(hipStreamSynchronize(ctx->stream));
    }
    t.gen = ++ctx->table_gen;
    *table_id = store_table(ctx->tables, std::move(t));
  });
}

int32_t prom_voigt_sigma(prom_ctx* ctx, int64_t n, const double* x, int32_t n_lines,
                         const double* line_wavelength, const double* line_gamma,
                         const double* line_coef, double sigma_v, double c_light, double* sigma_out) {
  return guarded(ctx, [&] {
    PROM_REQUIRE(sigma_out || n == 0, "prom_voigt_sigma: bad arguments");
    voigt_common(ctx, n, x, n_lines, line_wavelength, line_gamma, line_coef, ctx->scratch[0]);
    ctx->scratch[4].ensure(sizeof(double) * std::max<int64_t>(n, 1));
    prom::launch_voigt(ctx->stream, ctx->scratch[0].as<double>(), n, ctx->scratch[1].as<double>(),
                       ctx->scratch[2].as<double>(), ctx->scratch[3].as<double>(), n_lines, sigma_v, c_light,
                       0.0, 0, ctx->scratch[4].as<double>());
    download(sigma_out, ctx->scratch[4], n, ctx->stream);
    PROM_HIP(hipStreamSynchronize(ctx->stream));
  });
}

int32_t prom_table_lookup(prom_ctx* ctx, int32_t table_id, int64_t n_targets, const double* targets,
                          double* out) {
  return guarded(ctx, [&] {
    PROM_REQUIRE(table_ok(ctx->tables, table_id), "prom_table_lookup: unknown table");
    PROM_REQUIRE(n_targets >= 0 && (n_targets == 0 || (targets && out)), "prom_table_lookup: bad arguments");
    const prom::AtomTable& t = ctx->tables[table_id];
    upload(ctx->scratch[0], targets, n_targets, ctx->stream);
    ctx->scratch[1].ensure(sizeof(double) * std::max<int64_t>(n_targets, 1));
    prom::launch_table_lookup(ctx->stream, t.x.as<double>(), t.y.as<double>(), t.n, t.offset,
                              ctx->scratch[0].as<double>(), n_targets, ctx->scratch[1].as<double>());
    download(out, ctx->scratch[1], n_targets, ctx->stream);
    PROM_HIP(hipStreamSynchronize(ctx->stream));
  });
}

// A freed table's memory goes back to the device; a transit problem that reads it is invalidated.
static void free_table(prom_ctx* ctx, bool molecular, int32_t id) {
  for (auto st : ctx->streams) PROM_HIP(hipStreamSynchronize(st));   // runs in flight may read it
  prom::TransitDev& tr = ctx->tr;
  bool used = !molecular && tr.star && tr.star_table_id == id;
  for (const auto& t : tr.terms)
    if ((t.is_molecule != 0) == molecular && t.table == id) used = true;
  if (used) {
    drop_graphs(tr);
    tr.ready = false;
    tr.ran = false;
  }
  if (molecular) ctx->mtables[id] = prom::MolTable{};
  else ctx->tables[id] = prom::AtomTable{};
}

int32_t prom_table_free(prom_ctx* ctx, int32_t table_id) {
  return guarded(ctx, [&] {
    PROM_REQUIRE(table_ok(ctx->tables, table_id), "prom_table_free: unknown table");
    free_table(ctx, false, table_id);
  });
}

int32_t prom_molecular_free(prom_ctx* ctx, int32_t table_id) {
  return guarded(ctx, [&] {
    PROM_REQUIRE(table_ok(ctx->mtables, table_id), "prom_molecular_free: unknown table");
    free_table(ctx, true, table_id);
  });
}

int32_t prom_table_count(prom_ctx* ctx, int32_t* n_atomic, int32_t* n_molecular, int64_t* device_bytes) {
  return guarded(ctx, [&] {
    int32_t a = 0, m = 0;
    int64_t b = 0;
    for (const auto& t : ctx->tables)
      if (t.live) {
        ++a;
        b += (int64_t)(t.x.cap + t.y.cap + t.dir.cap + t.rec.cap);
      }
    for (const auto& t : ctx->mtables)
      if (t.live) {
        ++m;
        b += (int64_t)(t.P.cap + t.T.cap + t.W.cap + t.V.cap);
      }
    if (n_atomic) *n_atomic = a;
    if (n_molecular) *n_molecular = m;
    if (device_bytes) *device_bytes = b;
  });
}

// ------------------------------------------------------------------------------ molecular
int32_t prom_molecular_upload(prom_ctx* ctx, int32_t n_p, const double* P, int32_t n_t, const double* T,
                              int64_t n_w, const double* wavelength, const double* log_sigma,
                              double offset, int32_t* table_id) {
  return guarded(ctx, [&] {
    PROM_REQUIRE(n_p >= 2 && n_t >= 2 && n_w >= 2 && P && T && wavelength && log_sigma && table_id,
                 "prom_molecular_upload: bad arguments (each axis needs >= 2 nodes)");
    prom::MolTable t;
    upload(t.P, P, n_p, ctx->stream);
    upload(t.T, T, n_t, ctx->stream);
    upload(t.W, wavelength, n_w, ctx->stream);
    const int64_t nv = (int64_t)n_p * n_t * n_w;
    upload(t.V, log_sigma, nv, ctx->stream);
    t.n_p = n_p;
    t.n_t = n_t;
    t.n_w = n_w;
    t.offset = offset;
    double m = -INFINITY;
    for (int64_t i = 0; i < nv; ++i) m = std::max(m, log_sigma[i]);
    t.vmax = m;
    PROM_HIP(hipStreamSynchronize(ctx->stream));
    *table_id = store_table(ctx->mtables, std::move(t));
  });
}

int32_t prom_molecular_sigma(prom_ctx* ctx, int32_t table_id, int64_t n_chords, int32_t n_x,
                             const double* P, double T, int64_t n_wav, const double* wavelength,
                             double* sigma_out) {
  return guarded(ctx, [&] {
    PROM_REQUIRE(table_ok(ctx->mtables, table_id), "prom_molecular_sigma: unknown table");
    PROM_REQUIRE(n_chords >= 0 && n_x >= 0 && n_wav >= 0, "prom_molecular_sigma: bad sizes");
    const int64_t tot = n_chords * n_x * n_wav;
    upload(ctx->scratch[0], P, n_chords * n_x, ctx->stream);
    upload(ctx->scratch[1], wavelength, n_chords * n_wav, ctx->stream);
    ctx->scratch[2].ensure(sizeof(double) * std::max<int64_t>(tot, 1));
    prom::launch_molecular_sigma(ctx->stream, ctx->mtables[table_id], n_chords, n_x, ctx->scratch[0].as<double>(),
                                 T, n_wav, ctx->scratch[1].as<double>(), ctx->scratch[2].as<double>());
    download(sigma_out, ctx->scratch[2], tot, ctx->stream);
    PROM_HIP(hipStreamSynchronize(ctx->stream));
  });
}

// ------------------------------------------------------------------------------ density
int32_t prom_number_density(prom_ctx* ctx, const prom_density_model* model, int32_t n_x, const double* x,
                            int64_t n_chords, const double* y, const double* z, const double* body_x,
                            const double* body_y, double* n_out) {
  return guarded(ctx, [&] {
    PROM_REQUIRE(model && valid_kind(model->kind) && model->kind != PROM_DENSITY_TABULATED &&
                     model->kind != PROM_DENSITY_GRIDDED,
                 "prom_number_density: unknown, tabulated or gridded density kind (gridded: prom_gridded_density)");
    PROM_REQUIRE(n_x >= 0 && n_chords >= 0, "prom_number_density: bad sizes");
    upload(ctx->scratch[0], x, n_x, ctx->stream);
    upload(ctx->scratch[1], y, n_chords, ctx->stream);
    upload(ctx->scratch[2], z, n_chords, ctx->stream);
    upload(ctx->scratch[3], body_x, n_chords, ctx->stream);
    upload(ctx->scratch[4], body_y, n_chords, ctx->stream);
    ctx->scratch[5].ensure(sizeof(double) * std::max<int64_t>(n_chords * n_x, 1));
    prom::launch_density(ctx->stream, to_dev(*model), ctx->scratch[0].as<double>(), n_x,
                         ctx->scratch[1].as<double>(), ctx->scratch[2].as<double>(), ctx->scratch[3].as<double>(),
                         ctx->scratch[4].as<double>(), n_chords, ctx->scratch[5].as<double>());
    download(n_out, ctx->scratch[5], n_chords * n_x, ctx->stream);
    PROM_HIP(hipStreamSynchronize(ctx->stream));
  });
}

int32_t prom_gridded_density(prom_ctx* ctx, int32_t n_gx, const double* gx, int32_t n_gy, const double* gy,
                             int32_t n_gz, const double* gz, const double* values, int64_t n_points,
                             const double* px, const double* py, const double* pz, double* out) {
  return guarded(ctx, [&] {
    PROM_REQUIRE(n_gx >= 2 && n_gy >= 2 && n_gz >= 2 && gx && gy && gz && values,
                 "prom_gridded_density: need >= 2 nodes per axis");
    PROM_REQUIRE((int64_t)n_gx * n_gy * n_gz < ((int64_t)1 << 31), "prom_gridded_density: grid too large");
    PROM_REQUIRE(n_points >= 0 && (n_points == 0 || (px && py && pz && out)), "prom_gridded_density: bad points");
    for (const auto& ax : {std::make_pair(gx, n_gx), std::make_pair(gy, n_gy), std::make_pair(gz, n_gz)})
      for (int32_t i = 1; i < ax.second; ++i)
        PROM_REQUIRE(ax.first[i] > ax.first[i - 1], "prom_gridded_density: axes must be strictly ascending");
    const int64_t nv = (int64_t)n_gx * n_gy * n_gz;
    std::vector<double> g;
    g.reserve(n_gx + n_gy + n_gz + nv);
    g.insert(g.end(), gx, gx + n_gx);
    g.insert(g.end(), gy, gy + n_gy);
    g.insert(g.end(), gz, gz + n_gz);
    g.insert(g.end(), values, values + nv);
    upload(ctx->scratch[0], g.data(), (int64_t)g.size(), ctx->stream);
    upload(ctx->scratch[1], px, n_points, ctx->stream);
    upload(ctx->scratch[2], py, n_points, ctx->stream);
    upload(ctx->scratch[3], pz, n_points, ctx->stream);
    ctx->scratch[4].ensure(sizeof(double) * std::max<int64_t>(n_points, 1));
    prom::launch_gridded(ctx->stream, ctx->scratch[0].as<double>(), n_gx, n_gy, n_gz, n_points,
                         ctx->scratch[1].as<double>(), ctx->scratch[2].as<double>(), ctx->scratch[3].as<double>(),
                         ctx->scratch[4].as<double>());
    download(out, ctx->scratch[4], n_points, ctx->stream);
    PROM_HIP(hipStreamSynchronize(ctx->stream));
  });
}

// ------------------------------------------------------------------------------ transit
int32_t prom_transit_set(prom_ctx* ctx, const prom_transit_problem* pb) {
  return guarded(ctx, [&] {
    PROM_REQUIRE(pb, "prom_transit_set: null problem");
    prom::TransitDev& tr = ctx->tr;
    tr.ready = false;
    tr.ran = false;
    // sigma-segment cache key of this set (committed at the end, after the device copy succeeded)
    bool seg_key_new = false, seg_key_keep = false;
    std::vector<double> new_key_sh;
    std::vector<uint64_t> new_key_gen;
    PROM_REQUIRE(pb->n_wav >= 1 && pb->wavelength, "transit: need >= 1 wavelength");
    PROM_REQUIRE(pb->n_pr >= 1 && pb->n_orb >= 1 && pb->chord_y && pb->chord_z && pb->chord_fout,
                 "transit: need chords and phases");
    PROM_REQUIRE(pb->n_x >= 1 && pb->x, "transit: need line-of-sight samples");
    PROM_REQUIRE(pb->planet_y, "transit: planet_y missing");
    PROM_REQUIRE(pb->n_moons >= 0 && (pb->n_moons == 0 || (pb->moon_y && pb->moon_R)), "transit: moons");
    PROM_REQUIRE(pb->n_scenarios >= 1 && pb->scenarios, "transit: need >= 1 density scenario");
    PROM_REQUIRE(pb->n_wav <= ((int64_t)65535 << 8), "transit: n_wav too large for one shard");
    tr.n_wav = pb->n_wav;
    tr.n_pr = pb->n_pr;
    tr.n_orb = pb->n_orb;
    tr.n_x = pb->n_x;
    tr.n_sc = pb->n_scenarios;
    tr.n_moons = pb->n_moons;
    tr.delta_x = pb->delta_x;
    tr.planet_R = pb->planet_R;
    tr.cull_tau = pb->cull_tau > 0.0 ? pb->cull_tau : std::ldexp(1.0, -60);
    for (auto st : ctx->streams) PROM_HIP(hipStreamSynchronize(st));   // pipelined runs may still read the old problem
    drop_graphs(tr);   // captured against the old problem's buffers and arguments
    {
      // measured on MI355X (tools/host_overhead.py, C2): hipGraphLaunch costs the host ~16 us per run
      // against ~8.5 us for the three direct launches, so graphs are opt-in (PROM_GRAPH=1)
      const char* e = std::getenv("PROM_GRAPH");
      tr.graphs = e && std::atoi(e) != 0;
    }
    tr.exp_mode = (pb->options & PROM_OPT_OCML_EXP) ? 0 : 1;
    tr.merge = (pb->options & PROM_OPT_NO_MERGE) == 0;
    tr.window = (pb->options & PROM_OPT_NO_WINDOW) == 0;
    {
      const char* e = std::getenv("PROM_TAU_PLAN");
      tr.plan = !(e && std::atoi(e) == 0);
      const char* m = std::getenv("PROM_SPECIES_MERGE");
      tr.species_merge_ok = !(m && std::atoi(m) == 0);   // narrowed below
      const char* tc = std::getenv("PROM_TCURVE");
      tr.tcurve = !(tc && std::atoi(tc) == 0);            // narrowed below
      // the per-run switches of the windowed path, read here rather than in every prom_transit_run (getenv scans
      // the environment: ~1 us a call on the GPU box's hosts, against ~8.5 us for a run's three launches)
      const char* fk = std::getenv("PROM_SIGMA_FORK");
      tr.env_fork = fk ? (std::atoi(fk) != 0 ? 1 : 0) : -1;
      const char* sgs = std::getenv("PROM_SIG_STAGGER");
      tr.env_stagger = sgs && std::atoi(sgs) != 0;
    }
    PROM_REQUIRE(pb->n_pr < (1 << 24), "transit: n_pr must be < 2^24");
    tr.terms.clear();
    tr.dens.clear();
    tr.mslots.clear();
    tr.atom_sigma_max.clear();
    tr.tab_off.assign(tr.n_sc, -1);
    const hipStream_t s = ctx->stream;
    Stager stg;
    const int64_t n_orb = tr.n_orb;
    std::vector<double> bx(tr.n_sc * n_orb), by(tr.n_sc * n_orb), sh(tr.n_sc * n_orb);
    int64_t tab_total = 0;
    int32_t n_atoms = 0, n_mol = 0;
    for (int32_t sc = 0; sc < tr.n_sc; ++sc) {
      const prom_scenario& S = pb->scenarios[sc];
      PROM_REQUIRE(valid_kind(S.density.kind), "transit: unknown density kind");
      tr.dens.push_back(to_dev(S.density));
      PROM_REQUIRE(S.shift, "transit: scenario shift[] missing");
      if (S.density.kind == PROM_DENSITY_TABULATED) {
        PROM_REQUIRE(S.n_tabulated, "transit: tabulated scenario without n_tabulated");
        tr.tab_off[sc] = tab_total;
        tab_total += n_orb * tr.n_pr * tr.n_x;
      } else if (S.density.kind == PROM_DENSITY_GRIDDED) {
        int64_t gnx, gny, gnz, glen;
        PROM_REQUIRE(S.n_tabulated && gridded_dims(S.density, &gnx, &gny, &gnz, &glen),
                     "transit: gridded scenario needs p = {n_gx, n_gy, n_gz} (>= 2 each) and the packed grid");
        tr.tab_off[sc] = tab_total;
        tab_total += glen;
      } else {
        PROM_REQUIRE(S.body_x && S.body_y, "transit: scenario body position missing");
      }
      for (int64_t o = 0; o < n_orb; ++o) {
        bx[sc * n_orb + o] = S.body_x ? S.body_x[o] : 0.0;
        by[sc * n_orb + o] = S.body_y ? S.body_y[o] : 0.0;
        sh[sc * n_orb + o] = S.shift[o];
      }
      PROM_REQUIRE(S.n_constituents >= 0 && (S.n_constituents == 0 || S.constituents), "transit: constituents");
      for (int32_t k = 0; k < S.n_constituents; ++k) {
        const prom_constituent& C = S.constituents[k];
        prom::TermDev t{};
        t.scenario = sc;
        t.is_molecule = C.is_molecule ? 1 : 0;
        t.table = C.table_id;
        t.chi = C.chi;
        if (t.is_molecule) {
          PROM_REQUIRE(table_ok(ctx->mtables, C.table_id), "transit: unknown molecular table id");
          t.slot = n_mol++;
          const prom::MolTable& mt = ctx->mtables[C.table_id];
          prom::MolSlotDev md{};
          md.P = mt.P.as<double>(); md.T = mt.T.as<double>(); md.W = mt.W.as<double>(); md.V = mt.V.as<double>();
          md.n_p = mt.n_p; md.n_t = mt.n_t; md.n_w = mt.n_w;
          md.offset = mt.offset;
          md.fill = std::log10(mt.offset);
          md.temp = S.T;
          md.chi = C.chi;
          md.scenario = sc;
          tr.mslots.push_back(md);
        } else {
          PROM_REQUIRE(table_ok(ctx->tables, C.table_id), "transit: unknown table id");
          t.slot = n_atoms++;
          const prom::AtomTable& tb = ctx->tables[C.table_id];
          tr.atom_sigma_max.push_back((std::pow(10.0, tb.ymax) - tb.offset) * (1.0 + 1e-9));
        }
        tr.terms.push_back(t);
      }
    }
    tr.n_atoms = n_atoms;
    tr.n_mol = n_mol;
    tr.n_terms = (int32_t)tr.terms.size();
    // uploads
    stg.add(tr.wav, pb->wavelength, tr.n_wav, s);
    stg.add(tr.cy, pb->chord_y, tr.n_pr, s);
    stg.add(tr.cz, pb->chord_z, tr.n_pr, s);
    stg.add(tr.cfout, pb->chord_fout, tr.n_pr, s);
    {
      // mirror images (y, -z) of the chords, for k_mol_list's merging of equal molecular records: sorted by y,
      // each unpaired chord with z != 0 takes the first later chord within 1e-9 of (y, -z) (relative to its
      // radius); k_mol_list verifies the sample lists before merging anything
      const char* stg_env = std::getenv("PROM_MOL_STAGE");
      tr.mol_stage = !(stg_env && std::atoi(stg_env) == 0);
      const char* mir_env = std::getenv("PROM_MOL_MIRROR");
      const bool mir_on = !(mir_env && std::atoi(mir_env) == 0);
      tr.mirror_h.assign((size_t)tr.n_pr, -1);
      tr.n_mirror = 0;
      if (mir_on && tr.n_pr <= prom::kMolMirrorMax) {
        const double* cy = pb->chord_y;
        const double* cz = pb->chord_z;
        std::vector<int32_t> ord((size_t)tr.n_pr);
        for (int32_t i = 0; i < (int32_t)tr.n_pr; ++i) ord[i] = i;
        std::sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return cy[a] < cy[b] || (cy[a] == cy[b] && a < b); });
        for (size_t a = 0; a < ord.size(); ++a) {
          const int32_t i = ord[a];
          if (tr.mirror_h[i] >= 0 || !(cz[i] != 0.0) || !std::isfinite(cy[i]) || !std::isfinite(cz[i])) continue;
          const double tol = 1e-9 * std::max(std::fabs(cy[i]), std::fabs(cz[i]));
          for (size_t b = a + 1; b < ord.size() && cy[ord[b]] - cy[i] <= tol; ++b) {
            const int32_t j = ord[b];
            if (tr.mirror_h[j] < 0 && std::fabs(cz[j] + cz[i]) <= tol) {
              tr.mirror_h[i] = j;
              tr.mirror_h[j] = i;
              ++tr.n_mirror;
              break;
            }
          }
        }
      }
      stg.add(tr.mirror, tr.mirror_h.data(), tr.n_pr, s);
    }
    stg.add(tr.x, pb->x, tr.n_x, s);
    stg.add(tr.planet_y, pb->planet_y, n_orb, s);
    stg.add(tr.moon_y, pb->moon_y, (int64_t)tr.n_moons * n_orb, s);
    stg.add(tr.moon_R, pb->moon_R, tr.n_moons, s);
    stg.add(tr.body_x, bx.data(), (int64_t)bx.size(), s);
    stg.add(tr.body_y, by.data(), (int64_t)by.size(), s);
    stg.add(tr.shift, sh.data(), (int64_t)sh.size(), s);
    stg.add(tr.terms_dev, tr.terms.data(), (int64_t)tr.terms.size(), s);
    stg.add(tr.sigma_max_dev, tr.atom_sigma_max.data(), (int64_t)tr.atom_sigma_max.size(), s);
    {
      // the molecular tables at each slot's temperature, one 32-byte bilinear record per (P interval, lambda'
      // interval) (k_mol_gt: two 16-byte loads per sample in k_tau_mol)
      int64_t g_total = 0;
      for (const auto& md : tr.mslots) g_total += 2 * (int64_t)std::max(md.n_p - 1, 1) * (md.n_w - 1);
      if (g_total > 0) tr.mol_g.ensure(sizeof(double2) * (size_t)g_total);
      int64_t g_off = 0;
      for (auto& md : tr.mslots) {
        md.k_B = pb->k_B > 0.0 ? pb->k_B : 1.381 * std::pow(10.0, -16);
        md.shift = tr.shift.as<double>() + (int64_t)md.scenario * n_orb;
        md.G = tr.mol_g.as<double2>() + g_off;
        g_off += 2 * (int64_t)std::max(md.n_p - 1, 1) * (md.n_w - 1);
        prom::launch_mol_gt(s, md);
      }
    }
    stg.add(tr.molslot, tr.mslots.data(), (int64_t)tr.mslots.size(), s);
    {
      // per-scenario density bound n_ref (every built-in model peaks at p[0] = n_0 on its domain;
      // tabulated: the largest finite value) -> column normalisation c_s = 1 / (chi_s n_ref n_x dx)
      std::vector<double> nref(tr.n_sc, 0.0);
      for (int32_t sc = 0; sc < tr.n_sc; ++sc) {
        const prom_scenario& S = pb->scenarios[sc];
        if (S.density.kind == PROM_DENSITY_TABULATED) {
          double m = 0.0;
          const int64_t cnt = n_orb * tr.n_pr * tr.n_x;
          for (int64_t i = 0; i < cnt; ++i) {
            const double v = std::fabs(S.n_tabulated[i]);
            if (std::isfinite(v) && v > m) m = v;
          }
          nref[sc] = m;
        } else if (S.density.kind == PROM_DENSITY_GRIDDED) {
          // a trilinear value is a convex combination of corners (weights sum to 1 within rounding)
          int64_t gnx, gny, gnz, glen;
          gridded_dims(S.density, &gnx, &gny, &gnz, &glen);
          double m = 0.0;
          for (int64_t i = gnx + gny + gnz; i < glen; ++i) {
            const double v = std::fabs(S.n_tabulated[i]);
            if (std::isfinite(v) && v > m) m = v;
          }
          nref[sc] = m * (1.0 + 1e-9);
        } else {
          // p[0] bounds the built-in profile only where it decays away from its body: a growing power
          // law (q < 0), a negative scale height, a hydrostatic J_0 below J(R) or a negative n_0 would
          // make the normalised columns exceed 1 and the windows' envelopes under-estimate tau
          const double* p = S.density.p;
          bool bounded = p[0] >= 0.0 && std::isfinite(p[0]);
          if (S.density.kind == PROM_DENSITY_BAROMETRIC) bounded = bounded && p[2] > 0.0;
          if (S.density.kind == PROM_DENSITY_POWERLAW) bounded = bounded && p[2] >= 0.0 && p[1] > 0.0;
          if (S.density.kind == PROM_DENSITY_HYDROSTATIC)
            bounded = bounded && p[4] >= 0.0 && p[1] > 0.0 && p[3] != 0.0 &&
                      p[4] >= p[2] / (p[3] * p[1]) * (1.0 - 1e-12);
          if (!bounded) tr.window = false;
          nref[sc] = std::fabs(p[0]) * (1.0 + 1e-9);
        }
      }
      for (const auto& t : tr.terms)   // negative mixing ratios give negative columns: no envelopes
        if (!t.is_molecule && !(t.chi >= 0.0)) tr.window = false;
      std::vector<prom::SigTabDev> st;
      for (const auto& t : tr.terms) {
        if (t.is_molecule) continue;
        const prom::AtomTable& tb = ctx->tables[t.table];
        const double bound = std::fabs(t.chi) * nref[t.scenario] * (double)tr.n_x * tr.delta_x;
        const double c = (bound > 0.0 && std::isfinite(bound)) ? 1.0 / bound : 0.0;
        // an overflowing bound cannot normalise the columns: integrate without windows
        if (!std::isfinite(bound) || (bound > 0.0 && !(c > 0.0))) tr.window = false;
        const double inv = (c > 0.0 && std::isfinite(c)) ? bound : 0.0;
        st.push_back({tb.x.as<double>(), tb.y.as<double>(), tb.n, tb.offset,
                      tr.shift.as<double>() + (int64_t)t.scenario * n_orb, tb.dir.as<int32_t>(), tb.n_dir, 0,
                      tb.dir_x0, tb.dir_inv_h, std::isfinite(c) ? c : 0.0, inv, t.chi, tb.hx.front(), tb.hx.back(),
                      tb.rec.as<double4>()});
      }
      // species merging: one scenario carries every atomic constituent (and there are >= 2 of them)
      int32_t sc0 = -1;
      bool one_sc = n_atoms >= 2 && n_mol == 0;
      double smax_m = 0.0;
      for (const auto& t : tr.terms) {
        if (t.is_molecule) continue;
        if (sc0 < 0) sc0 = t.scenario;
        if (t.scenario != sc0 || !(std::isfinite(t.chi) && t.chi >= 0.0)) one_sc = false;
        smax_m += t.chi * tr.atom_sigma_max[t.slot];
      }
      tr.species_merge_ok = tr.species_merge_ok && one_sc && tr.n_sc <= 4;
      if (tr.species_merge_ok) {
        const double bound = nref[sc0] * (double)tr.n_x * tr.delta_x;
        const double c = (bound > 0.0 && std::isfinite(bound)) ? 1.0 / bound : 0.0;
        if (!std::isfinite(bound) || (bound > 0.0 && !(c > 0.0)) || !std::isfinite(smax_m)) tr.species_merge_ok = false;
        tr.sigtab_m = prom::SigTabs4{};
        tr.sigtab_m.t[0] = st[0];
        tr.sigtab_m.t[0].ncoef = std::isfinite(c) ? c : 0.0;
        tr.sigtab_m.t[0].nscale = (c > 0.0 && std::isfinite(c)) ? bound : 0.0;
        tr.sigtab_m.t[0].chi = 1.0;
        tr.colargs_m = prom::ColArgs{};
        prom::TermDev tm{};
        tm.scenario = sc0;
        tm.is_molecule = 0;
        tm.slot = 0;
        tm.table = -1;
        tm.chi = 1.0;
        tr.colargs_m.t[0] = tm;
        stg.add(tr.sigma_max_m, &smax_m, 1, s);
        tr.qbound_m = smax_m * tr.sigtab_m.t[0].nscale;
      }
      stg.add(tr.sigtab, st.data(), (int64_t)st.size(), s);
      tr.qbound_v = 0.0;
      for (size_t i = 0; i < st.size(); ++i) tr.qbound_v += tr.atom_sigma_max[i] * st[i].nscale;
      // transmission curves (prom_tcurve.hip): one effective absorber on the fast column path, windows allowed
      // (PROM_OPT_NO_WINDOW / OCML_EXP keep the exact validation paths), no stellar spectrum
      {
        const bool cols8e = n_mol == 0 && tr.n_x <= 64 && (int32_t)tr.terms.size() <= 8 && tr.n_sc <= 4;
        tr.tcurve = tr.tcurve && cols8e && tr.exp_mode && tr.window && !pb->has_star && n_atoms >= 1 &&
                    (n_atoms == 1 || tr.species_merge_ok);
        // Y bound (merged: sum_s chi_s sigma_max_s; one species: sigma_max) and the octave cap of the tables:
        // q = Y N_max <= Y_bound * (the column bound 1 / c), one octave of margin
        const double yb = !tr.tcurve ? 0.0 : (n_atoms == 1 ? tr.atom_sigma_max[0] : smax_m);
        const double nb = !tr.tcurve ? 0.0 : (n_atoms == 1 ? st[0].nscale : tr.sigtab_m.t[0].nscale);
        tr.tc_ybound = (std::isfinite(yb) && yb > 0.0) ? yb : 0.0;
        const double qb = yb * nb;
        int lg = prom::kTcMaxOctaves;
        if (std::isfinite(qb) && qb > 0.0) lg = std::max(1, std::min(prom::kTcMaxOctaves, std::ilogb(qb) + 7 + 2));
        // PROM_TC_LG (tests): a lower cap, so that points above the table take the exact per-point sum
        if (const char* e = std::getenv("PROM_TC_LG")) lg = std::max(1, std::min(lg, std::atoi(e)));
        tr.tc_lg = lg;
      }
      // PROM_OPT_DOPPLER_ROWS: one sigma row per phase even when the factors are equal (a phase shard of a
      // problem with orbital Doppler shift takes the full problem's sigma path: bitwise equal rows)
      tr.uniform_shift = !(pb->options & PROM_OPT_DOPPLER_ROWS);
      for (const auto& t : tr.terms) {
        if (t.is_molecule) continue;
        for (int64_t o = 1; o < n_orb; ++o)
          if (!(sh[t.scenario * n_orb + o] == sh[t.scenario * n_orb])) tr.uniform_shift = false;
      }
      tr.sigtab_v = prom::SigTabs4{};
      for (size_t i = 0; i < st.size() && i < 4; ++i) tr.sigtab_v.t[i] = st[i];
      // sigma segments of the Doppler rows (k_sigma_rows): per 256-wavelength block and atomic slot, nodes
      // [lo, hi] with X[lo] <= fl(s_min lambda_first) and fl(s_max lambda_last) < X[hi] (numpy's bracket j of
      // a target: the largest j <= n-2 with X[j] <= t), and a linear bracket guess verified over the slice
      tr.sig_seg_ok = false;
      std::vector<double> key_sh;
      std::vector<uint64_t> key_gen;
      for (const auto& t : tr.terms) {
        if (t.is_molecule) continue;
        key_gen.push_back(ctx->tables[t.table].gen);
        key_sh.insert(key_sh.end(), sh.begin() + t.scenario * n_orb, sh.begin() + (t.scenario + 1) * n_orb);
      }
      // (every path with resampled rows reads them, with or without orbital Doppler shift).  PROM_SIGMA_ROWS=0
      // (validation): every block without a guess -- per-target directory lookups (sigma_of) everywhere
      const char* srows = std::getenv("PROM_SIGMA_ROWS");
      const bool no_guess = srows && std::atoi(srows) == 0;
      // PROM_SEG_DIR=0 (comparisons): no bucket directories.  Like no_guess, such segments are neither reused nor
      // committed as the key, so toggling the switch between sets with the same tables never measures the other
      const char* e_sd = std::getenv("PROM_SEG_DIR");
      const bool use_dir = !(e_sd && std::atoi(e_sd) == 0);
      const bool want_seg = true;
      const bool seg_reuse = !no_guess && use_dir && tr.seg_key_valid && key_gen == tr.seg_key_gen &&
                             key_sh == tr.seg_key_sh && (int64_t)tr.seg_key_wav.size() == tr.n_wav &&
                             std::memcmp(tr.seg_key_wav.data(), pb->wavelength, sizeof(double) * tr.n_wav) == 0;
      // reused segments stay valid only if this set completes; a throw below must not leave the key
      // pointing at buffers a later (failed) set may have reallocated
      tr.seg_key_valid = false;
      seg_key_keep = seg_reuse;   // the stored key stays as it is (re-validated at the end)
      if (!seg_reuse) tr.tw_ok = false;
      // target windows (k_sigma_tw, prom_window.hip): every atomic slot on one set of Doppler factors (one scenario),
      // n_orb >= 2; built with the sigma segments (the same inputs) and kept when they are reused.  The default: C4x10
      // k_sigma_tw 47-48 us against k_sigma_tc's 60, pipelined step 0.062 against 0.065 ms; C3 (three merged species)
      // steps 0.0366-0.0374 against 0.0370-0.0384 ms on the same boxes, reads 46 against 79 MB per launch, though
      // 36-37 against 32 us isolated (profiles/r06t_*, r06u_*).  PROM_TW (read at every set): 0 never
      const char* e_tw = std::getenv("PROM_TW");
      const bool tw_off = e_tw && std::atoi(e_tw) == 0;
      auto build_tw = [&]() {
        tr.tw_ok = false;
        tr.n_tw = 0;
        std::vector<const std::vector<double>*> tabs;
        int32_t sc_tw = -1;
        bool one = n_orb >= 2;
        for (const auto& t : tr.terms) {
          if (t.is_molecule) continue;
          if (sc_tw < 0) sc_tw = t.scenario;
          for (int64_t o = 0; o < n_orb; ++o)
            if (!(sh[t.scenario * n_orb + o] == sh[sc_tw * n_orb + o])) one = false;
          tabs.push_back(&ctx->tables[t.table].hx);
        }
        if (!one || sc_tw < 0 || tw_off) return;
        // (profiling knobs, read once: wavelengths per row, points per window, LDS doubles per workgroup).  The point
        // cap scales with the rows: a window's wavelengths span its rows' Doppler spread (C4x10: ~600) on top of a row's
        // own, so many-phase windows of 64 wavelengths a row spend most of their staging there -- C4x10p128 1.07 ms per
        // step at 8,192 points, 0.67 ms at 32,768 (128 rows x 256), C4x10p64 0.40 / 0.34 ms (profiles/r06w_*)
        // wavelengths per row: 256, and up to 768 for few rows (a window's staging then serves more points): C4x10
        // (8 rows) 0.0605-0.0613 ms per step at 256, 0.0563-0.0575 at 512, 0.0544 at 768; C4 0.0118 / 0.0111-0.0113;
        // C4x10p64 (64 rows) 0.343 at 256, 0.366 at 512; C3 unchanged (its windows end at the LDS budget)
        static const int rowcap_env = [] { const char* e = std::getenv("PROM_TW_ROWCAP"); return e ? std::max(1, std::atoi(e)) : 0; }();
        const int rowcap = rowcap_env > 0 ? rowcap_env : std::max(256, std::min(768, (int)(4096 / std::max<int64_t>(1, n_orb)) / 64 * 64));
        static const int64_t pmax_env = [] { const char* e = std::getenv("PROM_TW_PMAX"); return e ? (int64_t)std::max(1, std::atoi(e)) : (int64_t)0; }();
        const int64_t pmax = pmax_env > 0 ? pmax_env : std::max<int64_t>(8192, (int64_t)rowcap * n_orb);
        static const int lamcap = [] {   // (wavelengths staged per window at most; 0: never)
          const char* e = std::getenv("PROM_TW_LAMCAP");
          return e ? std::max(0, std::min(prom::kTwLamCap, std::atoi(e))) : prom::kTwLamCap;
        }();
        static const int lds = [] {
          const char* e = std::getenv("PROM_TW_LDS");
          return e ? std::max(16, std::min(prom::kTwLds, std::atoi(e))) : prom::kTwLds;
        }();
        std::vector<prom::SigSeg> twseg;
        std::vector<int32_t> twrow, twlam;
        int32_t nw = 0;
        if (!prom::build_target_windows(pb->wavelength, tr.n_wav, sh.data() + (int64_t)sc_tw * n_orb, (int32_t)n_orb, tabs,
                                        lds, lamcap, rowcap, pmax, twseg, twrow, twlam, nw))
          return;
        stg.add(tr.tw_seg, twseg.data(), (int64_t)twseg.size(), s);
        stg.add(tr.tw_row, twrow.data(), (int64_t)twrow.size(), s);
        stg.add(tr.tw_lam, twlam.data(), (int64_t)twlam.size(), s);
        tr.n_tw = nw;
        tr.tw_ok = true;
        tr.tw_new = true;
        if (std::getenv("PROM_DEBUG")) {
          int64_t k[4] = {0, 0, 0, 0};
          for (const auto& e : twseg) k[e.kind & 3] += 1;
          int64_t lam_st = 0, lam_n = 0;   // windows whose wavelengths are staged; their wavelengths
          for (int32_t b = 0; b < nw; ++b)
            if (twlam[2 * b + 1] > twlam[2 * b]) {
              ++lam_st;
              lam_n += twlam[2 * b + 1] - twlam[2 * b];
            }
          std::fprintf(stderr, "[prom] target windows: %d (slices: %lld staged, %lld global, %lld staged unguessed, "
                       "%lld outside the table; wavelengths staged in %lld windows, %.1f per window)\n", nw,
                       (long long)k[1], (long long)k[2], (long long)k[3], (long long)k[0], (long long)lam_st,
                       lam_st ? (double)lam_n / (double)lam_st : 0.0);
        }
      };
      if (seg_reuse) {
        tr.sig_seg_ok = true;
        if (tw_off) tr.tw_ok = false;
        else if (!tr.tw_ok) build_tw();
      } else if (want_seg && n_atoms >= 1 && n_atoms <= 4) {
        tr.seg_key_valid = false;
        const int64_t nb = (tr.n_wav + prom::kSigBlockW - 1) / prom::kSigBlockW;
        std::vector<prom::SigSeg> seg(nb * n_atoms, prom::SigSeg{0, 0, 0, 0, 0.0, 0.0});
        std::vector<prom::SigSeg> seg4(nb * n_atoms * 4, prom::SigSeg{0, 0, 0, 0, 0.0, 0.0});   // per wavefront
        // bucket directories of blocks without a linear guess (their SigSeg appended to seg4 at the end, the
        // buckets in sig_dir); PROM_SEG_DIR=0 turns them off, for comparisons
        std::vector<prom::SigSeg> segr;
        std::vector<int32_t> sdir;
        std::mutex segr_mu;
        int32_t ia = 0;
        for (const auto& t : tr.terms) {
          if (t.is_molecule) continue;
          const prom::AtomTable& tb = ctx->tables[t.table];
          const std::vector<double>& X = tb.hx;
          const int64_t n = tb.n;
          double smin = INFINITY, smax = -INFINITY;
          bool ok = n >= 2 && (int64_t)X.size() == n;
          for (int64_t o = 0; o < n_orb; ++o) {
            const double v = sh[t.scenario * n_orb + o];
            if (!(v > 0.0) || !std::isfinite(v)) ok = false;
            smin = std::min(smin, v);
            smax = std::max(smax, v);
          }
          auto bracket = [&](double v) -> int64_t {
            int64_t j = (int64_t)(std::upper_bound(X.begin(), X.end(), v) - X.begin()) - 1;
            return j < 0 ? 0 : (j > n - 2 ? n - 2 : j);
          };
          // the slice [lo, hi] of targets in [tlo, thi] and its linear bracket guess, verified at both ends of
          // every node interval (g and numpy's bracket are monotone step functions, and the bracket is constant
          // inside an interval): kind 1 (LDS-sized) or 2 with a guess, 0 without; false: no slice
          auto make_seg = [&](double tlo, double thi, prom::SigSeg& e) -> bool {
            const int64_t lo = bracket(tlo);
            const int64_t hi = bracket(thi) + 1;
            const int64_t m = hi - lo + 1;
            if (m < 2 || m > INT32_MAX / 2) return false;
            e.lo = (int32_t)lo;
            e.m = (int32_t)m;
            const double xs = X[lo], span = X[hi] - X[lo];
            const double inv = span > 0.0 ? (double)(m - 1) / span : 0.0;
            const double b0 = -(xs * inv);
            bool lin = span > 0.0 && std::isfinite(inv) && std::isfinite(b0);
            auto guess = [&](double v) -> int64_t {
              const double f = std::fma(v, inv, b0);   // the device's seg_guess
              int64_t g = f < 0.0 ? 0 : (f >= (double)(m - 2) ? m - 2 : (int64_t)f);
              return g;
            };
            for (int64_t i = lo; lin && i < hi; ++i) {
              if (X[i] == X[i + 1]) continue;
              const double a = std::max(X[i], tlo), z = std::nextafter(X[i + 1], -INFINITY);
              if (a > z) continue;
              const int64_t k = i - lo;   // numpy's bracket on [X[i], X[i+1]) (i <= hi - 1 <= n - 2)
              const int64_t ga = guess(a), gz = guess(z);
              if (ga < k - 1 || ga > k + 1 || gz < k - 1 || gz > k + 1) lin = false;
            }
            e.kind = 0;
            if (lin) {
              e.kind = (m <= prom::kSigSeg ? 1 : 2) | (m <= prom::tc_slice_cap(n_atoms) ? 64 : 0);
              e.xs = b0;
              e.inv = inv;
            }
            return true;
          };
          auto blocks = [&](int64_t b0, int64_t b1) {
          for (int64_t b = b0; ok && b < b1; ++b) {
            double lmin = INFINITY, lmax = -INFINITY;
            bool fin = true;
            for (int64_t w = b * prom::kSigBlockW; w < std::min<int64_t>(tr.n_wav, (b + 1) * prom::kSigBlockW); ++w) {
              const double l = pb->wavelength[w];
              if (!(l > 0.0) || !std::isfinite(l)) fin = false;
              lmin = std::min(lmin, l);
              lmax = std::max(lmax, l);
            }
            if (!fin) continue;
            const double tlo = smin * lmin, thi = smax * lmax;
            // every target inside [x_0, x_{n-1}): no clamp or end rule
            if (!(tlo >= X[0] && thi < X[n - 1])) continue;
            prom::SigSeg& e = seg[b * n_atoms + ia];
            if (!make_seg(tlo, thi, e)) continue;
            if ((e.kind & 3) == 0) {
              // no guess over the block: one per wavefront of 64 wavelengths (oversize blocks read global
              // records per wavefront, so each wave may take its own slice and guess); m = 0: none for that wave
              bool any = false;
              for (int q = 0; q < prom::kSigBlockW / 64; ++q) {
                double wl = INFINITY, wh = -INFINITY;
                const int64_t w0 = b * prom::kSigBlockW + 64 * q;
                for (int64_t w = w0; w < std::min<int64_t>(tr.n_wav, w0 + 64); ++w) {
                  wl = std::min(wl, pb->wavelength[w]);
                  wh = std::max(wh, pb->wavelength[w]);
                }
                prom::SigSeg& ew = seg4[(b * n_atoms + ia) * 4 + q];
                if (wl <= wh && make_seg(smin * wl, smax * wh, ew) && (ew.kind & 3) != 0) {
                  ew.kind = 2;   // (read from the global records; never k_seg_exact's exact mark, never LDS)
                  any = true;
                } else {
                  ew = prom::SigSeg{0, 0, 0, 0, 0.0, 0.0};
                }
              }
              if (any) e.kind |= 8;
              // a slice whose node spacing varies too much for one linear guess: a bucket directory over the
              // slice (B uniform buckets, bucket j -> numpy's bracket at its start), verified within one node
              // of numpy's bracket at every target of the block; B = 4, 16, ..., 1024 times the slice's nodes (kind & 32; pad = its SigSeg in seg4 past the
              // per-wavefront entries, whose pad is the directory's offset in sig_dir)
              if (!use_dir) continue;
              const int64_t lo = e.lo, m = e.m, hi = lo + m - 1;
              const double x0 = X[lo], span = X[hi] - X[lo];
              if (!(span > 0.0)) continue;
              std::vector<int32_t> dv;
              prom::SigSeg de{(int32_t)lo, 0, 32, 0, 0.0, 0.0};
              bool okd = false;
              for (int64_t mult = 4; !okd && mult <= 1024 && m * mult <= (1 << 22); mult *= 4) {
                const int64_t B = m * mult;
                const double inv = (double)B / span, b0 = -(x0 * inv);
                if (!std::isfinite(inv) || !std::isfinite(b0)) break;
                dv.assign(B, 0);
                // bucket j starts at x0 + j span / B: the bracket there, by one sweep over the slice's nodes
                int64_t k = 0;
                for (int64_t j = 0; j < B; ++j) {
                  const double v = x0 + span * ((double)j / (double)B);
                  while (k < m - 2 && X[lo + k + 1] <= v) ++k;
                  dv[j] = (int32_t)k;
                }
                auto gd = [&](double v) -> int64_t {
                  const double f = std::fma(v, inv, b0);   // the device's seg_guess with m = B + 1
                  const int64_t j = f < 0.0 ? 0 : (f >= (double)(B - 1) ? B - 1 : (int64_t)f);
                  return dv[j];
                };
                // verified at the block's actual targets (every row's factor times every wavelength, the
                // kernel's clamped rows and lanes among them; the same products as the kernel's tt[]), so
                // node intervals no target falls in (near-coincident nodes) do not matter
                okd = true;
                for (int64_t o = 0; okd && o < n_orb; ++o) {
                  const double v = sh[t.scenario * n_orb + o];
                  for (int64_t w = b * prom::kSigBlockW; okd && w < (b + 1) * prom::kSigBlockW; ++w) {
                    const double tt = v * pb->wavelength[std::min<int64_t>(w, tr.n_wav - 1)];
                    const int64_t kk = bracket(tt) - lo, g = gd(tt);
                    if (kk < 0 || kk > m - 2 || g < kk - 1 || g > kk + 1) okd = false;
                  }
                }
                if (okd) {
                  de.m = (int32_t)(B + 1);
                  de.xs = b0;
                  de.inv = inv;
                }
              }
              if (okd) {
                std::lock_guard<std::mutex> lk(segr_mu);
                if (sdir.size() + dv.size() > ((size_t)1 << 26)) continue;   // (256 MB of directories at most)
                de.pad = (int32_t)sdir.size();
                e.pad = (int32_t)(seg4.size() + segr.size());
                segr.push_back(de);
                sdir.insert(sdir.end(), dv.begin(), dv.end());
                e.kind |= 32;
              }
            }
          }
          };
          // independent blocks: split over host threads (the guess verification visits every slice node)
          const int64_t n_thr = std::max<int64_t>(1, std::min<int64_t>(8, nb / 64));
          std::vector<std::thread> pool;
          for (int64_t t = 1; t < n_thr; ++t) pool.emplace_back(blocks, nb * t / n_thr, nb * (t + 1) / n_thr);
          blocks(0, nb / n_thr);
          for (auto& th : pool) th.join();
          ++ia;
        }
        if (no_guess)
          for (auto& e : seg) e.kind = 0;
        // (block, species) pairs left with neither a linear guess nor a directory (k_sigma_tc's front row split)
        tr.sig_noguess = 0;
        for (const auto& e : seg) tr.sig_noguess += (e.kind & 3) == 0 && !(e.kind & 32);
        stg.add(tr.sig_seg, seg.data(), (int64_t)seg.size(), s);
        seg4.insert(seg4.end(), segr.begin(), segr.end());
        stg.add(tr.sig_seg4, seg4.data(), (int64_t)seg4.size(), s);
        stg.add(tr.sig_dir, sdir.data(), (int64_t)sdir.size(), s);
        if (std::getenv("PROM_DEBUG"))
          std::fprintf(stderr, "[prom] bucket directories: %zu, %zu buckets\n", segr.size(), sdir.size());
        std::vector<int32_t> fbl, fbt;
        for (int64_t b = 0; b < nb; ++b) {
          bool lds = true, ldt = true;
          for (int32_t a = 0; a < n_atoms; ++a) {
            lds = lds && (seg[b * n_atoms + a].kind & ~64) == 1;
            ldt = ldt && (seg[b * n_atoms + a].kind & 64) != 0;
          }
          if (!lds) fbl.push_back((int32_t)b);
          if (!ldt) fbt.push_back((int32_t)b);
        }
        tr.n_sig_fb = (int32_t)fbl.size();
        tr.n_sig_fb_tc = (int32_t)fbt.size();
        if (fbl.empty()) fbl.push_back(0);
        if (fbt.empty()) fbt.push_back(0);
        stg.add(tr.sig_fb, fbl.data(), (int64_t)fbl.size(), s);
        stg.add(tr.sig_fb_tc, fbt.data(), (int64_t)fbt.size(), s);
        tr.sig_seg_ok = true;
        build_tw();
        // the key is committed only after the segments have reached the device (end of this call):
        // a set that throws later must not leave a key that a retry would reuse (validation segments never)
        seg_key_new = !no_guess && use_dir;
        new_key_sh = std::move(key_sh);
        new_key_gen = std::move(key_gen);
      }
    }
    // polynomial sigma rows: the smallest even degree D with amax^(D+1)/(D+1)! <= 2^-53 over the problem's
    // atomic tables (AtomTable::amax bounds |ln10 slope| h on every interval); 0 (exp10 rows) when a table
    // has non-finite values or |a| is too large for D <= 14
    tr.sig_deg = 0;
    {
      // PROM_SIG_POLY=0, and PROM_SIGMA_ROWS=0 (per-target directory lookups: numpy.interp + exp10 everywhere)
      const char* e = std::getenv("PROM_SIG_POLY");
      const char* er = std::getenv("PROM_SIGMA_ROWS");
      bool fin = !(e && std::atoi(e) == 0) && !(er && std::atoi(er) == 0);
      double am = 0.0;
      for (const auto& t : tr.terms) {
        if (t.is_molecule) continue;
        const double a = ctx->tables[t.table].amax;
        if (!(a == a)) fin = false;
        else am = std::max(am, a);
      }
      am *= 1.0 + 1e-6;
      for (int D = 4; fin && D <= 14; D += 2) {
        // Lagrange remainder relative to e^a: am^(D+1) / (D+1)! e^|a| (a < 0 carries the e^|a| factor)
        double term = std::exp(am);
        for (int i = 1; i <= D + 1; ++i) term *= am / (double)i;
        if (term <= std::ldexp(1.0, -53)) { tr.sig_deg = D; break; }
      }
    }
    tr.star = pb->has_star != 0;
    tr.star_table_id = tr.star ? pb->star_table : -1;
    if (tr.star) {
      // stellar spectrum: chord arrays, the F_star table and, per wavelength tile of the tau kernel, the
      // slice of table nodes its targets lambda / s_c can reach: s in [s_min, s_max] and IEEE division
      // is monotone, so fl(lambda / s) lies in [fl(lambda_min / s_max), fl(lambda_max / s_min)]
      PROM_REQUIRE(pb->chord_rho && pb->chord_clv && pb->chord_star_shift, "transit: stellar chord arrays missing");
      PROM_REQUIRE(table_ok(ctx->tables, pb->star_table), "transit: unknown star table id");
      PROM_REQUIRE(n_mol == 0 && n_atoms <= 8,
                   "transit: the stellar-spectrum path takes <= 8 atomic constituents and no molecules");
      const prom::AtomTable& sb = ctx->tables[pb->star_table];
      PROM_REQUIRE(sb.offset == 0.0, "transit: the star table must have offset 0 (n_interp_log(..., 0.0))");
      tr.star_tab = prom::SigTabDev{sb.x.as<double>(), sb.y.as<double>(), sb.n, sb.offset, nullptr,
                                    sb.dir.as<int32_t>(), sb.n_dir, 0, sb.dir_x0, sb.dir_inv_h, 0.0, 0.0, 0.0,
                                    sb.hx.front(), sb.hx.back(), sb.rec.as<double4>()};
      stg.add(tr.crho, pb->chord_rho, tr.n_pr, s);
      stg.add(tr.cclv, pb->chord_clv, tr.n_pr, s);
      stg.add(tr.cshift, pb->chord_star_shift, tr.n_pr, s);
      double smin = INFINITY, smax = -INFINITY;
      bool ok = sb.n >= 2 && (int64_t)sb.hx.size() == sb.n;
      for (int32_t i = 0; i < tr.n_pr; ++i) {
        const double v = pb->chord_star_shift[i];
        if (!(v > 0.0) || !std::isfinite(v)) ok = false;
        smin = std::min(smin, v);
        smax = std::max(smax, v);
      }
      tr.star_uniform = true;
      for (int32_t i = 1; i < tr.n_pr; ++i)
        if (!(pb->chord_star_shift[i] == pb->chord_star_shift[0])) tr.star_uniform = false;
      const int64_t n_tiles = (tr.n_wav + 255) / 256;
      std::vector<int32_t> sl(3 * n_tiles, 0);
      const std::vector<double>& X = sb.hx;
      const int64_t n = sb.n;
      auto bracket = [&](double t) -> int64_t {   // numpy's j: largest j <= n-2 with X[j] <= t (0 below)
        int64_t j = (int64_t)(std::upper_bound(X.begin(), X.end(), t) - X.begin()) - 1;
        return j < 0 ? 0 : (j > n - 2 ? n - 2 : j);
      };
      for (int64_t tl = 0; ok && tl < n_tiles; ++tl) {
        double lmin = INFINITY, lmax = -INFINITY;
        bool fin = true;
        for (int64_t w = tl * 256; w < std::min<int64_t>(tr.n_wav, (tl + 1) * 256); ++w) {
          const double l = pb->wavelength[w];
          if (!std::isfinite(l)) fin = false;
          lmin = std::min(lmin, l);
          lmax = std::max(lmax, l);
        }
        if (!fin) continue;
        const double tlo = lmin / smax, thi = lmax / smin;
        const int64_t lo = bracket(tlo);
        const int64_t hi = thi >= X[n - 1] ? n - 1 : bracket(thi) + 1;
        const int64_t m = hi - lo + 1;
        if (m < 2 || m > prom::kRmStarMax) continue;   // global lookups for this tile
        int32_t P = 1;
        while (P < m) P <<= 1;
        sl[3 * tl] = (int32_t)lo;
        sl[3 * tl + 1] = (int32_t)m;
        sl[3 * tl + 2] = P / 2;
      }
      stg.add(tr.rm_slices, sl.data(), (int64_t)sl.size(), s);
    }
    tr.tab.ensure(sizeof(double) * std::max<int64_t>(tab_total, 1));
    {
      std::vector<prom::ScDevHost> sd(tr.n_sc);
      for (int32_t sc = 0; sc < tr.n_sc; ++sc) {
        sd[sc].m = tr.dens[sc];
        sd[sc].tab = tr.tab_off[sc] >= 0 ? tr.tab.as<double>() + tr.tab_off[sc] : nullptr;
      }
      stg.add(tr.scdev, sd.data(), (int64_t)sd.size(), s);
      tr.colargs = prom::ColArgs{};
      for (int32_t i = 0; i < tr.n_sc && i < 4; ++i) tr.colargs.sc[i] = sd[i];
      for (int32_t i = 0; i < tr.n_sc && i < 4; ++i) tr.colargs_m.sc[i] = sd[i];
      for (int32_t i = 0; i < tr.n_terms && i < 8; ++i) tr.colargs.t[i] = tr.terms[i];
    }
    for (int32_t sc = 0; sc < tr.n_sc; ++sc)
      if (tr.tab_off[sc] >= 0) {
        int64_t len = n_orb * tr.n_pr * tr.n_x, gnx, gny, gnz;
        if (pb->scenarios[sc].density.kind == PROM_DENSITY_GRIDDED)
          gridded_dims(pb->scenarios[sc].density, &gnx, &gny, &gnz, &len);
        PROM_HIP(hipMemcpyAsync(tr.tab.as<double>() + tr.tab_off[sc], pb->scenarios[sc].n_tabulated,
                                sizeof(double) * len, hipMemcpyHostToDevice, s));
      }
    // work buffers
    const int64_t nc = n_orb * tr.n_pr;
    // pipelining needs every per-run buffer in the slot (n(c, x), the molecular samples and lists are); the
    // fast atomic paths and the molecular path run pipelined, the generic atomic column path (k_ntot +
    // k_columns: n_x > 64, > 8 terms or > 4 scenarios) and the stellar-spectrum path one slot
    const bool cols8 = n_mol == 0 && tr.n_x <= 64 && tr.n_terms <= 8 && tr.n_sc <= 4;
    const bool fast = tr.exp_mode && n_mol == 0 && n_atoms >= 1 && n_atoms <= prom::kWinMaxSpecies && tr.window &&
                      !tr.star && cols8;
    const bool mol_pipe = n_mol > 0 && !tr.star;
    tr.depth = (fast || mol_pipe) ? ctx->pipeline : 1;
    for (int si = 0; si < tr.depth; ++si) {
    prom::RunSlot& rs = tr.slot[si];
      if (!cols8) rs.ntot.ensure(sizeof(double) * tr.n_sc * nc * tr.n_x);
      rs.ncol.ensure(sizeof(double) * std::max<int64_t>(n_atoms, 1) * nc);
      rs.molcol.ensure(sizeof(double) * std::max<int64_t>(n_mol, 1) * nc);
      if (n_mol > 0) {
        rs.mol_smp.ensure(sizeof(double) * 4 * n_mol * nc * tr.n_x);
        rs.mol_nin.ensure(sizeof(int32_t) * n_mol * nc);
        rs.mol_lst.ensure(sizeof(double) * 4 * ((n_mol * tr.n_x + 1) * nc + (int64_t)prom::kMolListPad * n_orb));
        rs.mol_rend.ensure(sizeof(int32_t) * nc);
      }
      rs.flags.ensure(sizeof(int32_t) * nc);
      rs.recs.ensure(sizeof(double) * nc * (1 + n_atoms));
      rs.act_ip.ensure(sizeof(int32_t) * nc);
      rs.counts.ensure(sizeof(int32_t) * n_orb * prom::kCnt);
      rs.mrecs.ensure(sizeof(double) * nc * (1 + n_atoms));
      if (n_atoms >= 1 && n_atoms <= prom::kWinMaxSpecies && n_mol == 0) {
        rs.wenv.ensure(sizeof(int32_t) * n_orb * 2 * prom::kEnvN);
        rs.wmom.ensure(sizeof(double) * n_orb * (tr.n_pr + 1) *
                       std::max(prom::n_tail_moments(n_atoms), prom::n_tail_moments(1)));   // merged species: 1
      }
      rs.evals.ensure(sizeof(unsigned long long) * 64);
      // resampled cross-sections: one row per phase when the Doppler factors differ between phases
      const int64_t sig_rows = tr.uniform_shift ? 1 : n_orb;
      rs.sig.ensure(sizeof(double) * sig_rows * std::max<int64_t>(n_atoms, 1) * tr.n_wav);
      rs.zfl.ensure((size_t)(sig_rows * tr.n_wav));
      const int64_t n_wtiles = (tr.n_wav + 127) / 128;
      rs.tq.ensure(sizeof(float) * 4 * sig_rows * n_wtiles);

      rs.hlist.ensure(sizeof(int32_t) * 4 * 2 * n_orb * 2 * n_wtiles);   // small and big lists, <= 1 per half tile
      rs.hcnt.ensure(sizeof(int32_t) * 4);
      rs.trec.ensure(sizeof(int32_t) * 4 * n_orb * n_wtiles);   // {h, t, flags, 0} per (phase, tile)
      tr.taup_resident = 0;
      rs.tsum.ensure(sizeof(double) * n_orb);
      rs.fsum.ensure(sizeof(double) * n_orb);
      rs.R.ensure(sizeof(double) * n_orb * tr.n_wav);
      if (tr.tcurve) {
        // k_tc_build: ~300 chords per part (C3: 8 parts; profiles/r04h_tc_build_parts.txt), at most kTcPartMax
        // parts; one part needs no hand-off between workgroups; PROM_TC_PARTS (profiling) overrides
        tr.tc_parts = (int32_t)std::max<int64_t>(1, std::min<int64_t>(prom::kTcPartMax, (tr.n_pr + 299) / 300));
        if (const char* e = std::getenv("PROM_TC_PARTS"))
          if (std::atoi(e) > 0) tr.tc_parts = std::min(prom::kTcPartMax, std::atoi(e));
        {
          // the chords' F_out total (the disk sum's denominator, the same for every phase), in chord order
          double fsum = 0.0;
          for (int32_t i = 0; i < tr.n_pr; ++i) fsum += pb->chord_fout[i];
          tr.tc_fsum = fsum;
        }
        if (!tr.tc_const.p) {
          // c_k = sum_j f_j cm[k][j] at the nodes u_j = cos(pi (j + 1/2) / 16); node factors 2^((u_k + 1) / 2)
          std::vector<double> cc(prom::kTcD * prom::kTcD + prom::kTcD);
          for (int k = 0; k < prom::kTcD; ++k)
            for (int j = 0; j < prom::kTcD; ++j)
              cc[k * prom::kTcD + j] = std::cos(M_PI * (double)k * ((double)j + 0.5) / (double)prom::kTcD) *
                                       ((k == 0 ? 1.0 : 2.0) / (double)prom::kTcD);
          for (int k = 0; k < prom::kTcD; ++k)
            cc[prom::kTcD * prom::kTcD + k] = std::exp2(0.5 * (std::cos(M_PI * ((double)k + 0.5) / (double)prom::kTcD) + 1.0));
          tr.tc_const.ensure(sizeof(double) * cc.size());
          PROM_HIP(hipMemcpy(tr.tc_const.p, cc.data(), sizeof(double) * cc.size(), hipMemcpyHostToDevice));
        }
        const int64_t n_ch = (tr.tc_lg + prom::kTcChain - 1) / prom::kTcChain;
        rs.tc_hdr.ensure(sizeof(double) * n_orb * prom::kTcHdr);
        rs.tc_tab.ensure(sizeof(double) * n_orb * tr.tc_lg * prom::kTcD);
        rs.tc_part.ensure(sizeof(double) * n_orb * n_ch * prom::kTcPartMax * prom::kTcPartVals);
        const size_t cb = sizeof(int32_t) * n_orb * n_ch;
        if (rs.tc_cnt.cap < cb) {
          rs.tc_cnt.ensure(cb);
          PROM_HIP(hipMemsetAsync(rs.tc_cnt.p, 0, rs.tc_cnt.cap, s));
        }
        rs.tc_pp.ensure(sizeof(prom::TcPart) * (size_t)std::max<int64_t>(1, n_orb * (tr.n_pr / 32)));
      }
    }
    tr.last = 0;
    stg.flush(ctx, s);
    if (tr.star) prom::launch_rm_fout(s, tr);   // per set: the unocculted flux of every wavelength
    if (tr.tw_new) {
      // windows built by this call: mark the slices whose guess is numpy's bracket at every target (PROM_TW_EXACT=0:
      // never, for comparisons)
      const char* e_ex = std::getenv("PROM_TW_EXACT");
      if (!(e_ex && std::atoi(e_ex) == 0)) prom::launch_tw_exact(s, tr, n_atoms);
      tr.tw_new = false;
    }
    if (seg_key_new) {
      // segments built by this call: mark those whose guess is numpy's bracket for every target
      const int64_t nb = (tr.n_wav + prom::kSigBlockW - 1) / prom::kSigBlockW;
      tr.sig_flags.ensure(sizeof(int32_t) * nb * n_atoms);
      prom::launch_seg_exact(s, n_atoms, tr.sigtab_v, tr.wav.as<double>(), tr.n_wav, (int32_t)n_orb,
                             tr.sig_seg.as<prom::SigSeg>(), tr.sig_flags.as<int32_t>());
      if (std::getenv("PROM_DEBUG")) {
        std::vector<prom::SigSeg> hs(nb * n_atoms);
        PROM_HIP(hipMemcpyAsync(hs.data(), tr.sig_seg.p, sizeof(prom::SigSeg) * hs.size(), hipMemcpyDeviceToHost, s));
        PROM_HIP(hipStreamSynchronize(s));
        int64_t cnt[8] = {};
        for (const auto& e : hs) ++cnt[e.kind & 7];
        std::fprintf(stderr, "[prom] sigma segments: %lld blocks x %d species, %d oversize blocks (%d for k_sigma_tc), kinds: "
                     "none %lld, lds %lld, global %lld, lds exact %lld, global exact %lld; poly degree %d\n", (long long)nb,
                     n_atoms, tr.n_sig_fb, tr.n_sig_fb_tc, (long long)cnt[0], (long long)cnt[1], (long long)cnt[2],
                     (long long)cnt[5], (long long)cnt[6], tr.sig_deg);
      }
    }
    PROM_HIP(hipStreamSynchronize(s));
    if (seg_key_new) {
      tr.seg_key_wav.assign(pb->wavelength, pb->wavelength + tr.n_wav);
      tr.seg_key_sh = std::move(new_key_sh);
      tr.seg_key_gen = std::move(new_key_gen);
      tr.seg_key_valid = true;
    } else if (seg_key_keep) {
      tr.seg_key_valid = true;
    }
    tr.ready = true;
  });
}

int32_t prom_transit_run(prom_ctx* ctx, prom_transit_stats* stats) {
  return guarded(ctx, [&] {
    prom::TransitDev& tr = ctx->tr;
    if (!tr.ready) throw Error(PROM_E_STATE, "prom_transit_run: call prom_transit_set first");
    int variant = 0;
    hipEvent_t* ev = ctx->ev;
    const bool timed = ctx->timing && (ctx->window_runs++ % ctx->timing_stride) == 0;
    if (timed) {
      const size_t need = 4 * (size_t)(ctx->timed_runs + 1);
      while (ctx->tev.size() < need) {
        hipEvent_t e;
        PROM_HIP(hipEventCreate(&e));
        ctx->tev.push_back(e);
      }
      ev = &ctx->tev[4 * (size_t)ctx->timed_runs];
      constexpr int32_t kTsCap = 8192;   // workgroups a tau launch may stamp
      if (ctx->tsbuf.size() <= (size_t)ctx->timed_runs) {
        ctx->tsbuf.emplace_back();
        ctx->tsbuf.back().ensure(sizeof(unsigned long long) * 2 * kTsCap);
      }
      if (ctx->ts_blocks.size() <= (size_t)ctx->timed_runs) ctx->ts_blocks.resize(ctx->timed_runs + 1);
      ctx->tr.ts_out = ctx->tsbuf[ctx->timed_runs].as<unsigned long long>();
      ctx->tr.ts_cap = kTsCap;
      ctx->tr.ts_blocks = 0;
      ++ctx->timed_runs;
    }
    tr.count_evals = stats != nullptr;
    // pipelined problems alternate slots and streams: this run's column / ordering kernels overlap the
    // previous run's tau kernel; a slot is reused two runs later, after its stream's previous run
    const int si = (tr.last + 1) % tr.depth;
    const hipStream_t st = ctx->streams[si];
    prom::RunSlot& rs = tr.slot[si];
    // the slot's second stream: the one `depth` away (free when depth <= kMaxSlots / 2).  The fork shortens
    // one run (sigma rows beside k_columns8 / k_order) but costs pipelined throughput (C4 7.3e10 -> 3.8e10
    // pts/s, C3 unchanged: profiles/r02w_pipeline_sweep.txt), so it is the default for unpipelined
    // problems only; PROM_SIGMA_FORK=0/1 forces it off/on
    const bool fork_ok = tr.depth <= prom::kMaxSlots / 2 && (tr.env_fork >= 0 ? tr.env_fork != 0 : tr.depth == 1);
    rs.aux = fork_ok ? ctx->streams[si + tr.depth] : nullptr;
    rs.ev_fork = fork_ok ? ctx->fork_ev[si] : nullptr;
    rs.ev_join = fork_ok ? ctx->join_ev[si] : nullptr;
    // staggered kernel order on alternate slots (PROM_SIG_STAGGER=1): odd slots queue the Doppler sigma
    // rows after k_order, so their latency-bound ordering overlaps the even slots' full-chip kernels
    rs.sig_late = tr.depth > 1 && (si & 1) && tr.env_stagger;
    if (stats) PROM_HIP(hipMemsetAsync(rs.evals.p, 0, sizeof(unsigned long long) * 64, st));
    if (!stats && !timed && tr.graphs && tr.depth > 1) {
      // untimed fast-path run: replay the slot's graph (captured here the first time)
      if (!tr.gexec[si]) {
        hipGraph_t g = nullptr;
        PROM_HIP(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        try {
          prom::launch_transit(st, tr, rs, ctx->tables, ctx->mtables, nullptr, &variant, false);
        } catch (...) {
          (void)hipStreamEndCapture(st, &g);
          if (g) (void)hipGraphDestroy(g);
          throw;
        }
        PROM_HIP(hipStreamEndCapture(st, &g));
        const hipError_t ie = hipGraphInstantiate(&tr.gexec[si], g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        PROM_HIP(ie);
      }
      PROM_HIP(hipGraphLaunch(tr.gexec[si], st));
    } else {
      prom::launch_transit(st, tr, rs, ctx->tables, ctx->mtables, (stats || timed) ? ev : nullptr, &variant,
                           stats != nullptr);
    }
    tr.last = si;
    tr.count_evals = false;
    if (timed) ctx->ts_blocks[ctx->timed_runs - 1] = tr.ts_blocks;
    tr.ts_out = nullptr;
    tr.ts_blocks = 0;

    tr.ran = true;
    if (stats) {
      std::memset(stats, 0, sizeof(*stats));
      PROM_HIP(hipEventSynchronize(ev[3]));
      float a = 0, b = 0, c = 0, t = 0;
      PROM_HIP(hipEventElapsedTime(&a, ev[0], ev[1]));
      PROM_HIP(hipEventElapsedTime(&b, ev[1], ev[2]));
      PROM_HIP(hipEventElapsedTime(&c, ev[2], ev[3]));
      PROM_HIP(hipEventElapsedTime(&t, ev[0], ev[3]));
      stats->ms_density = a;
      stats->ms_sigma = b;
      stats->ms_tau = c;
      stats->ms_total = t;
      const int K = prom::kCnt;
      std::vector<int32_t> cnt(tr.n_orb * K);
      download(cnt.data(), rs.counts, (int64_t)cnt.size(), st);
      unsigned long long ev64[64];
      download(ev64, rs.evals, 64, st);
      PROM_HIP(hipStreamSynchronize(st));
      int64_t unwindowed = 0, counted = 0;
      for (int32_t o = 0; o < tr.n_orb; ++o) {
        const bool sorted = cnt[o * K + 5] != 0;
        const bool exact = cnt[o * K + 3] != 0;
        const int64_t recs = sorted ? cnt[o * K + 4] : cnt[o * K];
        stats->active_chords += cnt[o * K];
        stats->transparent_chords += cnt[o * K + 1];
        stats->blocked_chords += cnt[o * K + 2];
        stats->tau_records += recs;
        if (exact) stats->tau_kernel_variant_exact_phases += 1;
        // the device counters cover the non-exact phases of the atomic fast kernel
        if (exact || tr.n_mol > 0 || !tr.exp_mode || tr.n_atoms > prom::kWinMaxSpecies || tr.star) unwindowed += recs;
      }
      for (int i = 0; i < 64; ++i) counted += (int64_t)ev64[i];
      if (std::getenv("PROM_DEBUG") && rs.trec.p && rs.hcnt.p && rs.tq.p) {
        const int64_t n_wtiles = (tr.n_wav + 127) / 128;
        std::vector<int32_t> trv(4 * tr.n_orb * n_wtiles), hc(4);
        std::vector<float> tqv(4 * n_wtiles * tr.n_orb);
        download(trv.data(), rs.trec, (int64_t)trv.size(), st);
        download(hc.data(), rs.hcnt, 4, st);
        download(tqv.data(), rs.tq, (int64_t)tqv.size(), st);
        PROM_HIP(hipStreamSynchronize(st));
        long long win = 0, fl = 0;
        double tqs = 0.0;
        for (int64_t i = 0; i < tr.n_orb * n_wtiles; ++i) { win += trv[4 * i + 1] - trv[4 * i]; fl += trv[4 * i + 2]; }
        for (float v : tqv) tqs += v;
        std::fprintf(stderr, "prom: windows sum %lld flags sum %lld heavy small %d big %d tq sum %.9g\n", win, fl, hc[0],
                     hc[1], tqs);
        // heavy entries' record counts: small list, then big list (hcap = n_orb * 2 * n_tiles entries each)
        const int64_t hcap = (int64_t)tr.n_orb * 2 * n_wtiles;
        for (int b = 0; b < 2; ++b) {
          const int32_t ne = hc[b];
          if (ne <= 0 || !rs.hlist.p) continue;
          std::vector<int32_t> hl(4 * (size_t)ne);
          PROM_HIP(hipMemcpy(hl.data(), rs.hlist.as<int32_t>() + 4 * (b ? hcap : 0), sizeof(int32_t) * hl.size(),
                             hipMemcpyDeviceToHost));
          long long sum = 0;
          int32_t mx = 0;
          std::vector<int32_t> hist(8, 0);   // records: <=64, <=128, <=256, <=512, <=1024, <=2048, <=4096, more
          for (int32_t i = 0; i < ne; ++i) {
            const int32_t n = hl[4 * i + 2] - hl[4 * i + 1];
            sum += n;
            mx = std::max(mx, n);
            int k = 0;
            while (k < 7 && n > (64 << k)) ++k;
            ++hist[k];
          }
          std::fprintf(stderr, "prom: %s entries %d records sum %lld max %d  hist(<=64,128,..,4096,more) %d %d %d %d %d %d %d %d\n",
                       b ? "big" : "small", ne, sum, mx, hist[0], hist[1], hist[2], hist[3], hist[4], hist[5], hist[6],
                       hist[7]);
        }
      }
      if (std::getenv("PROM_DEBUG"))
        for (int32_t o = 0; o < tr.n_orb; ++o)
          std::fprintf(stderr, "prom: phase %d active %d records %d candidates %d sort %d largest slot %d\n", o,
                       cnt[o * K], cnt[o * K + 4], cnt[o * K + 7] & 8191, (cnt[o * K + 7] >> 13) & 3,
                       cnt[o * K + 7] >> 16);
      stats->chord_lambda_evals = stats->active_chords * tr.n_wav;
      stats->exp_evals = counted + unwindowed * tr.n_wav;
      stats->tau_kernel_variant = variant;
    }
  });
}

int32_t prom_transit_kernel_ms(prom_ctx* ctx, int32_t n_runs, double* ms_out) {
  return guarded(ctx, [&] {
    prom::TransitDev& tr = ctx->tr;
    if (!tr.ready) throw Error(PROM_E_STATE, "prom_transit_kernel_ms: call prom_transit_set first");
    PROM_REQUIRE(n_runs >= 1 && ms_out, "prom_transit_kernel_ms: bad arguments");
    for (auto st : ctx->streams) PROM_HIP(hipStreamSynchronize(st));
    std::vector<hipEvent_t> ev(2 * PROM_K_COUNT);
    for (auto& e : ev) PROM_HIP(hipEventCreate(&e));
    std::vector<double> sum(PROM_K_COUNT, 0.0);
    std::vector<int32_t> cnt(PROM_K_COUNT, 0);
    const hipStream_t st = ctx->streams[0];
    prom::RunSlot& rs = tr.slot[0];
    rs.aux = nullptr;
    rs.ev_fork = rs.ev_join = nullptr;
    rs.sig_late = false;
    int variant = 0;
    try {
      for (int32_t r = 0; r < n_runs; ++r) {
        tr.kprof = ev.data();
        tr.kprof_mask = 0;
        prom::launch_transit(st, tr, rs, ctx->tables, ctx->mtables, nullptr, &variant, false);
        tr.kprof = nullptr;
        PROM_HIP(hipStreamSynchronize(st));
        for (int k = 0; k < PROM_K_COUNT; ++k) {
          if (!(tr.kprof_mask & (1u << k))) continue;
          float ms = 0.0f;
          PROM_HIP(hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]));
          sum[k] += ms;
          ++cnt[k];
        }
      }
    } catch (...) {
      tr.kprof = nullptr;
      for (auto e : ev) (void)hipEventDestroy(e);
      throw;
    }
    for (auto e : ev) PROM_HIP(hipEventDestroy(e));
    tr.last = 0;
    tr.ran = true;
    for (int k = 0; k < PROM_K_COUNT; ++k) ms_out[k] = cnt[k] ? sum[k] / cnt[k] : std::nan("");
  });
}

int32_t prom_transit_result(prom_ctx* ctx, double* R_out) {
  return guarded(ctx, [&] {
    prom::TransitDev& tr = ctx->tr;
    if (!tr.ran) throw Error(PROM_E_STATE, "prom_transit_result: no completed run");
    PROM_REQUIRE(R_out, "prom_transit_result: null output");
    for (auto st : ctx->streams) PROM_HIP(hipStreamSynchronize(st));
    const size_t bytes = sizeof(double) * (size_t)tr.n_orb * (size_t)tr.n_wav;
    const char* src = static_cast<const char*>(tr.slot[tr.last].R.p);
    if (pinned_pool().holds(R_out, bytes)) {
      // page-locked destination (prom_host_alloc): DMA straight into it, split over PROM_D2H_SPLIT streams
      const char* e = std::getenv("PROM_D2H_SPLIT");
      const size_t k = (size_t)std::max(1, std::min(prom::kMaxSlots, e ? std::atoi(e) : 1));
      const size_t part = ((bytes + k - 1) / k + 4095) & ~(size_t)4095;
      for (size_t i = 0; i < k && i * part < bytes; ++i)
        PROM_HIP(hipMemcpyAsync(reinterpret_cast<char*>(R_out) + i * part, src + i * part,
                                std::min(part, bytes - i * part), hipMemcpyDeviceToHost, ctx->streams[i]));
      for (size_t i = 0; i < k; ++i) PROM_HIP(hipStreamSynchronize(ctx->streams[i]));
      return;
    }
    // D2H in chunks into pinned staging (one DMA per chunk, full link rate) while host threads copy the
    // finished chunks out to the caller's (pageable) array: the copy-out overlaps the transfer and runs on
    // several cores instead of one
    constexpr size_t kChunk = (size_t)2 << 20;
    const size_t n_chunks = (bytes + kChunk - 1) / kChunk;
    if (ctx->pin_cap < bytes) {
      if (ctx->pin) PROM_HIP(hipHostFree(ctx->pin));
      ctx->pin = nullptr;
      ctx->pin_cap = 0;
      PROM_HIP(hipHostMalloc(&ctx->pin, bytes, hipHostMallocDefault));
      ctx->pin_cap = bytes;
    }
    while (ctx->pin_ev.size() < n_chunks) {
      hipEvent_t e;
      PROM_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      ctx->pin_ev.push_back(e);
    }
    char* pin = static_cast<char*>(ctx->pin);
    for (size_t c = 0; c < n_chunks; ++c) {
      const size_t off = c * kChunk, len = std::min(kChunk, bytes - off);
      PROM_HIP(hipMemcpyAsync(pin + off, src + off, len, hipMemcpyDeviceToHost, ctx->stream));
      PROM_HIP(hipEventRecord(ctx->pin_ev[c], ctx->stream));
    }
    const size_t n_thr = std::min<size_t>(n_chunks, 8);
    std::vector<hipError_t> errs(n_thr, hipSuccess);
    auto copier = [&](size_t t) {
      for (size_t c = t; c < n_chunks; c += n_thr) {
        const hipError_t e = hipEventSynchronize(ctx->pin_ev[c]);
        if (e != hipSuccess) { errs[t] = e; return; }
        const size_t off = c * kChunk, len = std::min(kChunk, bytes - off);
        std::memcpy(reinterpret_cast<char*>(R_out) + off, pin + off, len);
      }
    };
    std::vector<std::thread> pool;
    for (size_t t = 1; t < n_thr; ++t) pool.emplace_back(copier, t);
    copier(0);
    for (auto& th : pool) th.join();
    for (auto e : errs) PROM_HIP(e);
  });
}

int32_t prom_transit_columns(prom_ctx* ctx, double* N_out) {
  return guarded(ctx, [&] {
    prom::TransitDev& tr = ctx->tr;
    if (!tr.ran) throw Error(PROM_E_STATE, "prom_transit_columns: no completed run");
    PROM_REQUIRE(N_out, "prom_transit_columns: null output");
    for (auto st : ctx->streams) PROM_HIP(hipStreamSynchronize(st));
    download(N_out, tr.slot[tr.last].ncol, (int64_t)tr.n_atoms * tr.n_orb * tr.n_pr, ctx->stream);
    PROM_HIP(hipStreamSynchronize(ctx->stream));
  });
}

int32_t prom_transit_band_stats(prom_ctx* ctx, int32_t n_bands, const double* bounds, double* sum_out,
                                int64_t* count_out, double* max_out) {
  return guarded(ctx, [&] {
    prom::TransitDev& tr = ctx->tr;
    if (!tr.ran) throw Error(PROM_E_STATE, "prom_transit_band_stats: no completed run");
    PROM_REQUIRE(n_bands >= 0 && (n_bands == 0 || bounds) && sum_out && count_out && max_out,
                 "prom_transit_band_stats: bad arguments");
    const int32_t n_orb = tr.n_orb;
    // the last run's stream orders the reduction after it; scratch[0..2] are free between calls
    const hipStream_t st = ctx->streams[tr.last];
    upload(ctx->scratch[0], bounds, (int64_t)n_orb * n_bands * 2, st);
    ctx->scratch[1].ensure(sizeof(double) * n_orb);
    ctx->scratch[2].ensure(sizeof(int64_t) * n_orb);
    ctx->scratch[3].ensure(sizeof(double) * n_orb);
    prom::launch_band_stats(st, tr.slot[tr.last].R.as<double>(), tr.wav.as<double>(), n_orb, tr.n_wav, n_bands,
                            ctx->scratch[0].as<double>(), ctx->scratch[1].as<double>(),
                            ctx->scratch[2].as<int64_t>(), ctx->scratch[3].as<double>());
    download(sum_out, ctx->scratch[1], n_orb, st);
    download(count_out, ctx->scratch[2], n_orb, st);
    download(max_out, ctx->scratch[3], n_orb, st);
    PROM_HIP(hipStreamSynchronize(st));
  });
}

int32_t prom_star_disk_flux(prom_ctx* ctx, int32_t star_table, int32_t n_cells, const double* shift,
                            const double* clv, const double* rho, double dphi, double drho, int64_t n_wav,
                            const double* wavelength, double* out) {
  return guarded(ctx, [&] {
    PROM_REQUIRE(table_ok(ctx->tables, star_table), "prom_star_disk_flux: unknown star table");
    PROM_REQUIRE(n_cells >= 0 && n_wav >= 0 && (n_cells == 0 || (shift && clv && rho)) &&
                     (n_wav == 0 || (wavelength && out)),
                 "prom_star_disk_flux: bad arguments");
    const prom::AtomTable& sb = ctx->tables[star_table];
    PROM_REQUIRE(sb.offset == 0.0, "prom_star_disk_flux: the star table must have offset 0 (10**Fstar_function)");
    // interp1d(bounds_error=True) semantics of the reference's Fstar_function: every target lambda / shift
    // inside [x_0, x_{n-1}] (IEEE division is monotone: the extremes decide)
    double smin = INFINITY, smax = -INFINITY, lmin = INFINITY, lmax = -INFINITY;
    for (int32_t c = 0; c < n_cells; ++c) {
      PROM_REQUIRE(shift[c] > 0.0 && std::isfinite(shift[c]), "prom_star_disk_flux: Doppler factors must be positive");
      smin = std::min(smin, shift[c]);
      smax = std::max(smax, shift[c]);
    }
    for (int64_t w = 0; w < n_wav; ++w) {
      PROM_REQUIRE(std::isfinite(wavelength[w]), "prom_star_disk_flux: non-finite wavelength");
      lmin = std::min(lmin, wavelength[w]);
      lmax = std::max(lmax, wavelength[w]);
    }
    if (n_cells > 0 && n_wav > 0) {
      PROM_REQUIRE(lmin / smax >= sb.hx.front(), "prom_star_disk_flux: a target is below the interpolation range");
      PROM_REQUIRE(lmax / smin <= sb.hx.back(), "prom_star_disk_flux: a target is above the interpolation range");
    }
    const prom::SigTabDev tb{sb.x.as<double>(), sb.y.as<double>(), sb.n, sb.offset, nullptr, sb.dir.as<int32_t>(),
                             sb.n_dir, 0, sb.dir_x0, sb.dir_inv_h, 0.0, 0.0, 0.0, sb.hx.front(), sb.hx.back(),
                             sb.rec.as<double4>()};
    const hipStream_t s = ctx->stream;
    upload(ctx->scratch[0], shift, n_cells, s);
    upload(ctx->scratch[1], clv, n_cells, s);
    upload(ctx->scratch[2], rho, n_cells, s);
    upload(ctx->scratch[3], wavelength, n_wav, s);
    ctx->scratch[4].ensure(sizeof(double) * std::max<int64_t>(n_wav, 1));
    prom::launch_star_disk(s, tb, ctx->scratch[0].as<double>(), ctx->scratch[1].as<double>(),
                           ctx->scratch[2].as<double>(), n_cells, dphi, drho, ctx->scratch[3].as<double>(), n_wav,
                           ctx->scratch[4].as<double>());
    download(out, ctx->scratch[4], n_wav, s);
    PROM_HIP(hipStreamSynchronize(s));
  });
}

int32_t prom_timing_begin(prom_ctx* ctx) {
  return guarded(ctx, [&] {
    ctx->timing = true;
    ctx->timed_runs = 0;
    ctx->window_runs = 0;
  });
}

int32_t prom_timing_stride(prom_ctx* ctx, int32_t stride) {
  return guarded(ctx, [&] {
    PROM_REQUIRE(stride >= 1, "prom_timing_stride: stride must be >= 1");
    ctx->timing_stride = stride;
  });
}

int32_t prom_timing_end(prom_ctx* ctx, int32_t max_runs, double* ms, int32_t* n_runs) {
  return guarded(ctx, [&] {
    PROM_REQUIRE(n_runs && (max_runs <= 0 || ms), "prom_timing_end: bad arguments");
    ctx->timing = false;
    const int32_t n = std::min(ctx->timed_runs, std::max(max_runs, 0));
    for (auto st : ctx->streams) PROM_HIP(hipStreamSynchronize(st));
    int clock_khz = 0;
    PROM_HIP(hipDeviceGetAttribute(&clock_khz, hipDeviceAttributeWallClockRate, ctx->device));
    std::vector<unsigned long long> ts;
    for (int32_t r = 0; r < n; ++r) {
      hipEvent_t* e = &ctx->tev[4 * (size_t)r];
      float v[4];
      // timed runs carry one event pair: the ordering kernel's completion -> the tau kernel's
      // completion (the tau kernel's run time plus its dispatch behind the ordering kernel)
      PROM_HIP(hipEventElapsedTime(&v[2], e[2], e[3]));
      ms[4 * r + 0] = ms[4 * r + 1] = ms[4 * r + 3] = std::nan("");
      ms[4 * r + 2] = v[2];
      // and the tau kernel's own span on the device clock: first workgroup start -> last workgroup end
      const int32_t nb = r < (int32_t)ctx->ts_blocks.size() ? ctx->ts_blocks[r] : 0;
      if (nb > 0 && clock_khz > 0) {
        ts.resize(2 * (size_t)nb);
        PROM_HIP(hipMemcpy(ts.data(), ctx->tsbuf[r].p, sizeof(unsigned long long) * ts.size(), hipMemcpyDeviceToHost));
        unsigned long long lo = ~0ull, hi = 0;
        for (int32_t b = 0; b < nb; ++b) {
          lo = std::min(lo, ts[2 * (size_t)b]);
          hi = std::max(hi, ts[2 * (size_t)b + 1]);
        }
        if (hi >= lo) ms[4 * r + 3] = (double)(hi - lo) / (double)clock_khz;
      }
    }
    *n_runs = ctx->timed_runs;
    ctx->timed_runs = 0;
  });
}

}  // extern "C"
