// Native input pipeline (host side) — the framework's replacement for the tf.data C++ runtime the
// reference reaches through list_files / decode_png / resize / cache / shuffle / batch / prefetch
// (reference dist_model_tf_vgg.py:34-65, fed_model.py:65-96,
// secure_fed_model.py:173-204).
//
//   decode_pngs(paths, size, out, threads)  PNG -> RGB8 -> TF2-style bilinear resize (half-pixel
//                                           centres, no antialias) into a uint8 NHWC array, on a
//                                           pool of worker threads (libpng, GIL released).
//   shuffle_order(index, buffer, seed)      tf.data shuffle-buffer order (a window of `buffer`
//                                           elements, uniform pick, refill from the stream).
//   BatchLoader                             prefetching batch assembler: worker threads gather the
//                                           rows of upcoming batches into a ring of caller-owned
//                                           (pinned) host slots; the consumer takes the slots in
//                                           batch order and hands each back after its H2D copy.
//
// Host-only C++17 + libpng, no HIP: the device side of the pipeline is one non_blocking copy from a
// pinned slot followed by the plan's input-staging kernel (csrc/kernels/nn_kernels.hip).
#include <png.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <csetjmp>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

// ------------------------------------------------------------------------------------------ PNG
struct PngImage {
  int w = 0, h = 0;
  std::vector<uint8_t> rgb;  // h*w*3
};

// Decode any PNG colour type / bit depth to 8-bit RGB (tf.io.decode_png(channels=3)).
// Everything libpng touches after setjmp lives in `ctx` (no automatic objects with destructors
// between setjmp and a longjmp out of libpng).
bool read_png(const std::string& path, PngImage& img, std::string& err) {
  struct Ctx {
    FILE* f = nullptr;
    png_structp png = nullptr;
    png_infop info = nullptr;
    png_bytep* rows = nullptr;
    ~Ctx() {
      if (png) png_destroy_read_struct(&png, info ? &info : nullptr, nullptr);
      if (f) fclose(f);
      delete[] rows;
    }
  } ctx;
  ctx.f = fopen(path.c_str(), "rb");
  if (!ctx.f) {
    err = "cannot open " + path;
    return false;
  }
  uint8_t sig[8];
  if (fread(sig, 1, 8, ctx.f) != 8 || png_sig_cmp(sig, 0, 8)) {
    err = "not a PNG: " + path;
    return false;
  }
  ctx.png = png_create_read_struct(PNG_LIBPNG_VER_STRING, nullptr, nullptr, nullptr);
  if (!ctx.png) {
    err = "png_create_read_struct failed";
    return false;
  }
  ctx.info = png_create_info_struct(ctx.png);
  if (!ctx.info) {
    err = "png_create_info_struct failed";
    return false;
  }
  if (setjmp(png_jmpbuf(ctx.png))) {
    err = "corrupt PNG: " + path;
    return false;
  }
  png_init_io(ctx.png, ctx.f);
  png_set_sig_bytes(ctx.png, 8);
  png_read_info(ctx.png, ctx.info);
  const int ct = png_get_color_type(ctx.png, ctx.info);
  const int bd = png_get_bit_depth(ctx.png, ctx.info);
  if (ct == PNG_COLOR_TYPE_PALETTE) png_set_palette_to_rgb(ctx.png);
  if (ct == PNG_COLOR_TYPE_GRAY && bd < 8) png_set_expand_gray_1_2_4_to_8(ctx.png);
  if (png_get_valid(ctx.png, ctx.info, PNG_INFO_tRNS)) png_set_tRNS_to_alpha(ctx.png);
  if (bd == 16) png_set_strip_16(ctx.png);
  if (ct == PNG_COLOR_TYPE_GRAY || ct == PNG_COLOR_TYPE_GRAY_ALPHA) png_set_gray_to_rgb(ctx.png);
  png_set_strip_alpha(ctx.png);
  png_read_update_info(ctx.png, ctx.info);
  const int w = (int)png_get_image_width(ctx.png, ctx.info);
  const int h = (int)png_get_image_height(ctx.png, ctx.info);
  const size_t rb = png_get_rowbytes(ctx.png, ctx.info);
  if (w <= 0 || h <= 0 || rb != (size_t)w * 3) {
    err = "unexpected PNG layout: " + path;
    return false;
  }
  img.w = w;
  img.h = h;
  img.rgb.resize((size_t)h * rb);
  ctx.rows = new png_bytep[h];
  for (int y = 0; y < h; ++y) ctx.rows[y] = img.rgb.data() + (size_t)y * rb;
  png_read_image(ctx.png, ctx.rows);
  png_read_end(ctx.png, nullptr);
  return true;
}

// tf.image.resize(method='bilinear', antialias=False) (TF2: half-pixel centres, edge clamp),
// evaluated on the decoded intensities and rounded back to uint8 for the cached NHWC array.
void resize_bilinear(const PngImage& src, int S, uint8_t* dst) {
  if (src.w == S && src.h == S) {
    std::memcpy(dst, src.rgb.data(), (size_t)S * S * 3);
    return;
  }
  const float sy = (float)src.h / S, sx = (float)src.w / S;
  for (int y = 0; y < S; ++y) {
    const float fy = (y + 0.5f) * sy - 0.5f;
    const int yf = (int)std::floor(fy);
    const float wy = fy - yf;
    const int y0 = std::min(std::max(yf, 0), src.h - 1);
    const int y1 = std::min(std::max(yf + 1, 0), src.h - 1);
    for (int x = 0; x < S; ++x) {
      const float fx = (x + 0.5f) * sx - 0.5f;
      const int xf = (int)std::floor(fx);
      const float wx = fx - xf;
      const int x0 = std::min(std::max(xf, 0), src.w - 1);
      const int x1 = std::min(std::max(xf + 1, 0), src.w - 1);
      const uint8_t* p00 = &src.rgb[((size_t)y0 * src.w + x0) * 3];
      const uint8_t* p01 = &src.rgb[((size_t)y0 * src.w + x1) * 3];
      const uint8_t* p10 = &src.rgb[((size_t)y1 * src.w + x0) * 3];
      const uint8_t* p11 = &src.rgb[((size_t)y1 * src.w + x1) * 3];
      for (int c = 0; c < 3; ++c) {
        const float top = p00[c] + (p01[c] - p00[c]) * wx;
        const float bot = p10[c] + (p11[c] - p10[c]) * wx;
        const float v = top + (bot - top) * wy;
        dst[((size_t)y * S + x) * 3 + c] = (uint8_t)std::lround(std::min(std::max(v, 0.f), 255.f));
      }
    }
  }
}

template <class F>
void parallel_for(size_t n, int threads, F&& fn) {
  threads = std::max(1, std::min<int>(threads, (int)std::max<size_t>(n, 1)));
  std::atomic<size_t> next{0};
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(1)) < n;) fn(i);
    });
  for (auto& th : pool) th.join();
}

// Returns (index, message) for every file that failed to decode (its rows are zero-filled).
std::vector<std::pair<int64_t, std::string>> decode_pngs(const std::vector<std::string>& paths, int size,
                                                          py::array_t<uint8_t, py::array::c_style> out,
                                                          int threads) {
  auto buf = out.request(true);
  if (buf.ndim != 4 || buf.shape[0] != (py::ssize_t)paths.size() || buf.shape[1] != size ||
      buf.shape[2] != size || buf.shape[3] != 3)
    throw std::invalid_argument("out must be uint8 [len(paths), size, size, 3]");
  uint8_t* base = static_cast<uint8_t*>(buf.ptr);
  const size_t per = (size_t)size * size * 3;
  std::vector<std::string> errs(paths.size());
  {
    py::gil_scoped_release nogil;
    parallel_for(paths.size(), threads, [&](size_t i) {
      PngImage img;
      std::string err;
      uint8_t* dst = base + i * per;
      if (read_png(paths[i], img, err)) {
        resize_bilinear(img, size, dst);
      } else {
        std::memset(dst, 0, per);
        errs[i] = err;
      }
    });
  }
  std::vector<std::pair<int64_t, std::string>> bad;
  for (size_t i = 0; i < errs.size(); ++i)
    if (!errs[i].empty()) bad.emplace_back((int64_t)i, errs[i]);
  return bad;
}

// ------------------------------------------------------------------------------------ shuffle
// splitmix64-seeded xoshiro256** with Lemire's unbiased bounded draw
struct Rng {
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    for (auto& v : s) {
      seed += 0x9E3779B97F4A7C15ull;
      uint64_t z = seed;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      v = z ^ (z >> 31);
    }
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  uint64_t below(uint64_t n) {
    unsigned __int128 m = (unsigned __int128)next() * n;
    uint64_t l = (uint64_t)m;
    if (l < n) {
      const uint64_t t = (0 - n) % n;
      while (l < t) {
        m = (unsigned __int128)next() * n;
        l = (uint64_t)m;
      }
    }
    return (uint64_t)(m >> 64);
  }
};

py::array_t<int64_t> shuffle_order(py::array_t<int64_t, py::array::c_style | py::array::forcecast> index,
                                   int64_t buffer, uint64_t seed) {
  auto in = index.request();
  const int64_t n = in.shape[0];
  const int64_t* src = static_cast<const int64_t*>(in.ptr);
  py::array_t<int64_t> out(n);
  int64_t* dst = static_cast<int64_t*>(out.request().ptr);
  Rng rng(seed);
  if (buffer >= n) {  // the window covers the whole stream: a uniform permutation
    std::copy(src, src + n, dst);
    for (int64_t i = n - 1; i > 0; --i) std::swap(dst[i], dst[rng.below((uint64_t)i + 1)]);
    return out;
  }
  std::vector<int64_t> pool(src, src + std::max<int64_t>(buffer, 1));
  int64_t j = (int64_t)pool.size();
  for (int64_t i = 0; i < n; ++i) {
    const int64_t k = (int64_t)rng.below(pool.size());
    dst[i] = pool[k];
    if (j < n) {
      pool[k] = src[j++];
    } else {
      pool[k] = pool.back();
      pool.pop_back();
    }
  }
  return out;
}

// ---------------------------------------------------------------------------------- BatchLoader
// Ring of `nslots` caller-owned host slots (x: batch*row_bytes, y: batch*label_bytes).  Batch b of
// the current epoch lives in slot b % nslots; a worker fills it once the consumer has released
// the slot's previous batch.  The consumer must release every taken slot before start_epoch().
class BatchLoader {
 public:
  BatchLoader(py::array x, py::array y, int64_t batch, std::vector<uintptr_t> xslots,
              std::vector<uintptr_t> yslots, int threads)
      : x_(x), y_(y), batch_(batch), xs_(std::move(xslots)), ys_(std::move(yslots)) {
    if (!(x.flags() & py::array::c_style) || !(y.flags() & py::array::c_style))
      throw std::invalid_argument("x and y must be C-contiguous");
    if (xs_.size() != ys_.size() || xs_.empty()) throw std::invalid_argument("need matching x/y slots");
    if (batch_ < 1) throw std::invalid_argument("batch must be >= 1");
    n_ = x.shape(0);
    if (y.shape(0) != n_) throw std::invalid_argument("x/y length mismatch");
    row_ = n_ ? (int64_t)x.nbytes() / n_ : 0;
    lab_ = n_ ? (int64_t)y.nbytes() / n_ : 0;
    xp_ = static_cast<const uint8_t*>(x.data());
    yp_ = static_cast<const uint8_t*>(y.data());
    nslots_ = (int64_t)xs_.size();
    state_.assign(nslots_, kFree);
    sizes_.assign(nslots_, 0);
    slot_batch_.assign(nslots_, -1);
    for (int t = 0; t < std::max(1, threads); ++t) workers_.emplace_back([this] { work(); });
  }
  ~BatchLoader() { shutdown(); }

  void shutdown() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (stop_) return;
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_)
      if (t.joinable()) t.join();
  }

  // Begin an epoch over `order` (dataset row indices); unconsumed batches of the previous epoch
  // are dropped.
  void start_epoch(py::array_t<int64_t, py::array::c_style | py::array::forcecast> order, bool drop_remainder) {
    auto o = order.request();
    const int64_t* op = static_cast<const int64_t*>(o.ptr);
    std::vector<int64_t> ord(op, op + o.shape[0]);
    for (int64_t v : ord)
      if (v < 0 || v >= n_) throw std::out_of_range("order index out of range");
    py::gil_scoped_release nogil;
    std::unique_lock<std::mutex> lk(mu_);
    for (int s : state_)
      if (s == kTaken) throw std::runtime_error("release every taken slot before start_epoch");
    cv_.wait(lk, [&] { return busy_ == 0; });  // no worker still copying into a slot
    order_ = std::move(ord);
    const int64_t n = (int64_t)order_.size();
    nbatches_ = drop_remainder ? n / batch_ : (n + batch_ - 1) / batch_;
    next_fill_ = next_take_ = 0;
    ++epoch_;
    std::fill(state_.begin(), state_.end(), (int)kFree);
    std::fill(slot_batch_.begin(), slot_batch_.end(), -1);
    lk.unlock();
    cv_.notify_all();
  }

  // Block until the next batch is ready: (slot, rows), or (-1, 0) after the last batch.
  std::pair<int64_t, int64_t> next() {
    py::gil_scoped_release nogil;
    std::unique_lock<std::mutex> lk(mu_);
    if (next_take_ >= nbatches_) return {-1, 0};
    const int64_t b = next_take_;
    const int64_t s = b % nslots_;
    cv_.wait(lk, [&] { return stop_ || (state_[s] == kReady && slot_batch_[s] == b); });
    if (stop_) return {-1, 0};
    state_[s] = kTaken;
    ++next_take_;
    return {s, sizes_[s]};
  }

  // The consumer is done with `slot` (its H2D copy has completed); the slot may be refilled.
  void release(int64_t slot) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (slot < 0 || slot >= nslots_ || state_[slot] != kTaken) throw std::invalid_argument("bad slot");
      state_[slot] = kFree;
    }
    cv_.notify_all();
  }

  int64_t num_batches() const { return nbatches_; }
  int64_t num_slots() const { return nslots_; }

 private:
  enum : int { kFree = 0, kFilling = 1, kReady = 2, kTaken = 3 };

  void work() {
    std::unique_lock<std::mutex> lk(mu_);
    while (true) {
      // batch b may only enter slot b % nslots once that slot is free (its previous batch,
      // b - nslots, was taken and released)
      cv_.wait(lk, [&] {
        return stop_ || (next_fill_ < nbatches_ && next_fill_ < next_take_ + nslots_ &&
                         state_[next_fill_ % nslots_] == kFree);
      });
      if (stop_) return;
      const int64_t b = next_fill_++;
      const int64_t s = b % nslots_;
      state_[s] = kFilling;
      slot_batch_[s] = b;
      ++busy_;
      const int64_t lo = b * batch_;
      const int64_t hi = std::min<int64_t>(lo + batch_, (int64_t)order_.size());
      const int64_t* ord = order_.data();
      lk.unlock();
      uint8_t* xd = reinterpret_cast<uint8_t*>(xs_[s]);
      uint8_t* yd = reinterpret_cast<uint8_t*>(ys_[s]);
      for (int64_t i = lo; i < hi; ++i) {
        const int64_t r = ord[i];
        std::memcpy(xd + (i - lo) * row_, xp_ + r * row_, row_);
        std::memcpy(yd + (i - lo) * lab_, yp_ + r * lab_, lab_);
      }
      lk.lock();
      --busy_;
      sizes_[s] = hi - lo;
      state_[s] = kReady;
      cv_.notify_all();
    }
  }

  py::array x_, y_;  // keep the source arrays alive
  const uint8_t* xp_ = nullptr;
  const uint8_t* yp_ = nullptr;
  int64_t n_ = 0, row_ = 0, lab_ = 0, batch_ = 1, nslots_ = 0;
  std::vector<uintptr_t> xs_, ys_;
  std::vector<int64_t> order_;
  std::vector<int> state_;
  std::vector<int64_t> sizes_, slot_batch_;
  int64_t nbatches_ = 0, next_fill_ = 0, next_take_ = 0, epoch_ = 0;
  int busy_ = 0;
  bool stop_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::thread> workers_;
};

}  // namespace

PYBIND11_MODULE(_idc_data, m) {
  m.doc() = "idc_models_amd native input pipeline (PNG decode/resize, shuffle buffer, prefetching batcher)";
  m.def("decode_pngs", &decode_pngs, py::arg("paths"), py::arg("size"), py::arg("out"), py::arg("threads") = 8);
  m.def("shuffle_order", &shuffle_order, py::arg("index"), py::arg("buffer"), py::arg("seed"));
  py::class_<BatchLoader>(m, "BatchLoader")
      .def(py::init<py::array, py::array, int64_t, std::vector<uintptr_t>, std::vector<uintptr_t>, int>(),
           py::arg("x"), py::arg("y"), py::arg("batch"), py::arg("xslots"), py::arg("yslots"),
           py::arg("threads") = 2)
      .def("start_epoch", &BatchLoader::start_epoch, py::arg("order"), py::arg("drop_remainder") = false)
      .def("next", &BatchLoader::next)
      .def("release", &BatchLoader::release)
      .def("shutdown", &BatchLoader::shutdown)
      .def_property_readonly("num_batches", &BatchLoader::num_batches)
      .def_property_readonly("num_slots", &BatchLoader::num_slots);
}
