// Paillier homomorphic encryption over GMP — the parity mode of secure aggregation.
//
// The reference protects the first ⌊n_tensors·percent⌋ weight tensors with `phe` Paillier
// (secure_fed_model.py:32,79,109-129): every weight is encrypted on the client,
// the server multiplies ciphertexts (= adds plaintexts) and divides by the client count, every
// client decrypts.  Encryption and decryption are one modular exponentiation per element with a
// 3072-bit modulus, so this is the hot loop of that path; here it runs on GMP (mpz_powm) across
// C++ threads with the GIL released, instead of Python big-int `pow`.
//
//   encrypt(n, m[int64], threads)            c = (1 + m·n) · r^n  mod n²   (g = n + 1), r ← getrandom
//   add(n, a, b)                             a·b mod n²  (element-wise homomorphic sum)
//   decrypt(p, q, c, threads) -> int64       CRT decryption mod p² and q² (≈4× fewer limb ops than
//                                            c^λ mod n²); signed result in (-n/2, n/2]
//
// Ciphertexts cross the boundary as ONE fixed-width big-endian byte block per element
// (width = bytes(n²)), i.e. a uint8 [count, width] numpy array.
#include <gmp.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

struct Mpz {
  mpz_t v;
  Mpz() { mpz_init(v); }
  ~Mpz() { mpz_clear(v); }
  Mpz(const Mpz&) = delete;
  Mpz& operator=(const Mpz&) = delete;
};

void from_bytes(mpz_t out, const uint8_t* p, size_t len) { mpz_import(out, len, 1, 1, 1, 0, p); }

void to_bytes(const mpz_t x, uint8_t* p, size_t width) {
  const size_t need = (mpz_sizeinbase(x, 2) + 7) / 8;
  if (need > width) throw std::runtime_error("value wider than the ciphertext width");
  std::memset(p, 0, width);
  size_t cnt = 0;
  mpz_export(p + (width - need), &cnt, 1, 1, 1, 0, x);
}

void mpz_from_pybytes(mpz_t out, const py::bytes& b) {
  std::string s = b;
  from_bytes(out, reinterpret_cast<const uint8_t*>(s.data()), s.size());
}

void random_bytes(uint8_t* p, size_t len) {
  while (len) {
    ssize_t got = getrandom(p, len, 0);
    if (got < 0) throw std::runtime_error("getrandom failed");
    p += got;
    len -= (size_t)got;
  }
}

template <class F>
void parallel_for(size_t n, int threads, F&& fn) {
  threads = std::max(1, std::min<int>(threads, (int)std::max<size_t>(n, 1)));
  std::atomic<size_t> next{0};
  std::vector<std::thread> pool;
  std::vector<std::string> errs(threads);
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      try {
        for (size_t i; (i = next.fetch_add(1)) < n;) fn(i);
      } catch (const std::exception& e) {
        errs[t] = e.what();
        next = n;
      }
    });
  for (auto& th : pool) th.join();
  for (auto& e : errs)
    if (!e.empty()) throw std::runtime_error(e);
}

size_t width_for(const mpz_t n) {
  Mpz n2;
  mpz_mul(n2.v, n, n);
  return (mpz_sizeinbase(n2.v, 2) + 7) / 8;
}

py::array_t<uint8_t> encrypt(py::bytes n_be, py::array_t<int64_t, py::array::c_style | py::array::forcecast> m,
                             int threads) {
  Mpz n, n2;
  mpz_from_pybytes(n.v, n_be);
  if (mpz_cmp_ui(n.v, 3) < 0) throw std::invalid_argument("bad modulus");
  mpz_mul(n2.v, n.v, n.v);
  const size_t W = width_for(n.v);
  const size_t nb = (mpz_sizeinbase(n.v, 2) + 7) / 8;
  auto mb = m.request();
  const int64_t cnt = mb.shape[0];
  const int64_t* mv = static_cast<const int64_t*>(mb.ptr);
  py::array_t<uint8_t> out({(py::ssize_t)cnt, (py::ssize_t)W});
  uint8_t* op = static_cast<uint8_t*>(out.request().ptr);
  {
    py::gil_scoped_release nogil;
    parallel_for((size_t)cnt, threads, [&](size_t i) {
      Mpz r, g, c, mm;
      std::vector<uint8_t> rb(nb + 16);
      // r uniform in [1, n) with gcd(r, n) = 1 (overwhelmingly likely on the first draw)
      do {
        random_bytes(rb.data(), rb.size());
        from_bytes(r.v, rb.data(), rb.size());
        mpz_mod(r.v, r.v, n.v);
        mpz_gcd(g.v, r.v, n.v);
      } while (mpz_cmp_ui(r.v, 0) == 0 || mpz_cmp_ui(g.v, 1) != 0);
      mpz_powm(c.v, r.v, n.v, n2.v);  // r^n mod n^2
      // g^m = 1 + m·n (mod n^2) for g = n + 1; negative m encoded as m mod n
      mpz_set_si(mm.v, (long)mv[i]);
      mpz_mod(mm.v, mm.v, n.v);
      mpz_mul(mm.v, mm.v, n.v);
      mpz_add_ui(mm.v, mm.v, 1);
      mpz_mul(c.v, c.v, mm.v);
      mpz_mod(c.v, c.v, n2.v);
      to_bytes(c.v, op + i * W, W);
    });
  }
  return out;
}

py::array_t<uint8_t> add(py::bytes n_be, py::array_t<uint8_t, py::array::c_style> a,
                         py::array_t<uint8_t, py::array::c_style> b) {
  Mpz n, n2;
  mpz_from_pybytes(n.v, n_be);
  mpz_mul(n2.v, n.v, n.v);
  const size_t W = width_for(n.v);
  auto ab = a.request(), bb = b.request();
  if (ab.ndim != 2 || bb.ndim != 2 || ab.shape[0] != bb.shape[0] || (size_t)ab.shape[1] != W ||
      (size_t)bb.shape[1] != W)
    throw std::invalid_argument("ciphertext blocks must be uint8 [count, width(n^2)] of equal count");
  const int64_t cnt = ab.shape[0];
  py::array_t<uint8_t> out({(py::ssize_t)cnt, (py::ssize_t)W});
  uint8_t* op = static_cast<uint8_t*>(out.request().ptr);
  const uint8_t* ap = static_cast<const uint8_t*>(ab.ptr);
  const uint8_t* bp = static_cast<const uint8_t*>(bb.ptr);
  py::gil_scoped_release nogil;
  Mpz x, y;
  for (int64_t i = 0; i < cnt; ++i) {
    from_bytes(x.v, ap + i * W, W);
    from_bytes(y.v, bp + i * W, W);
    mpz_mul(x.v, x.v, y.v);
    mpz_mod(x.v, x.v, n2.v);
    to_bytes(x.v, op + i * W, W);
  }
  return out;
}

// h_p = L_p(g^(p-1) mod p^2)^-1 mod p with g = n + 1
void crt_half(const mpz_t p, const mpz_t n, mpz_t p2, mpz_t h) {
  Mpz g, e;
  mpz_mul(p2, p, p);
  mpz_add_ui(g.v, n, 1);
  mpz_sub_ui(e.v, p, 1);
  mpz_powm(h, g.v, e.v, p2);
  mpz_sub_ui(h, h, 1);
  mpz_divexact(h, h, p);
  if (mpz_invert(h, h, p) == 0) throw std::invalid_argument("key is not invertible (bad p/q)");
}

py::array_t<int64_t> decrypt(py::bytes p_be, py::bytes q_be, py::array_t<uint8_t, py::array::c_style> c,
                             int threads) {
  Mpz p, q, n, p2, q2, hp, hq, qinv, half;
  mpz_from_pybytes(p.v, p_be);
  mpz_from_pybytes(q.v, q_be);
  mpz_mul(n.v, p.v, q.v);
  crt_half(p.v, n.v, p2.v, hp.v);
  crt_half(q.v, n.v, q2.v, hq.v);
  if (mpz_invert(qinv.v, q.v, p.v) == 0) throw std::invalid_argument("p and q not coprime");
  mpz_fdiv_q_2exp(half.v, n.v, 1);
  const size_t W = width_for(n.v);
  auto cb = c.request();
  if (cb.ndim != 2 || (size_t)cb.shape[1] != W) throw std::invalid_argument("ciphertext width mismatch");
  const int64_t cnt = cb.shape[0];
  const uint8_t* cp = static_cast<const uint8_t*>(cb.ptr);
  py::array_t<int64_t> out(cnt);
  int64_t* op = static_cast<int64_t*>(out.request().ptr);
  {
    py::gil_scoped_release nogil;
    parallel_for((size_t)cnt, threads, [&](size_t i) {
      Mpz x, mp, mq, e, t;
      from_bytes(x.v, cp + i * W, W);
      // m_p = L_p(c^(p-1) mod p^2) * h_p mod p  (and the same mod q)
      mpz_sub_ui(e.v, p.v, 1);
      mpz_mod(t.v, x.v, p2.v);
      mpz_powm(mp.v, t.v, e.v, p2.v);
      mpz_sub_ui(mp.v, mp.v, 1);
      mpz_divexact(mp.v, mp.v, p.v);
      mpz_mul(mp.v, mp.v, hp.v);
      mpz_mod(mp.v, mp.v, p.v);
      mpz_sub_ui(e.v, q.v, 1);
      mpz_mod(t.v, x.v, q2.v);
      mpz_powm(mq.v, t.v, e.v, q2.v);
      mpz_sub_ui(mq.v, mq.v, 1);
      mpz_divexact(mq.v, mq.v, q.v);
      mpz_mul(mq.v, mq.v, hq.v);
      mpz_mod(mq.v, mq.v, q.v);
      // CRT: m = m_q + q * ((m_p - m_q) * q^-1 mod p)
      mpz_sub(t.v, mp.v, mq.v);
      mpz_mul(t.v, t.v, qinv.v);
      mpz_mod(t.v, t.v, p.v);
      mpz_mul(t.v, t.v, q.v);
      mpz_add(t.v, t.v, mq.v);
      if (mpz_cmp(t.v, half.v) > 0) mpz_sub(t.v, t.v, n.v);
      if (!mpz_fits_slong_p(t.v)) throw std::overflow_error("plaintext does not fit int64");
      op[i] = (int64_t)mpz_get_si(t.v);
    });
  }
  return out;
}

// base^exp mod mod (big-endian byte strings): the finite-field Diffie-Hellman key agreement of
// mask-based secure aggregation (idc_models_amd/fed/keyagree.py) — constant-time mpz_powm_sec
// for the secret exponent
py::bytes powm(py::bytes base_be, py::bytes exp_be, py::bytes mod_be) {
  Mpz b, e, md, r;
  mpz_from_pybytes(b.v, base_be);
  mpz_from_pybytes(e.v, exp_be);
  mpz_from_pybytes(md.v, mod_be);
  if (mpz_cmp_ui(md.v, 3) < 0 || mpz_even_p(md.v)) throw std::invalid_argument("modulus must be odd and > 2");
  {
    py::gil_scoped_release nogil;
    if (mpz_sgn(e.v) > 0) mpz_powm_sec(r.v, b.v, e.v, md.v);
    else mpz_set_ui(r.v, 1);
  }
  const size_t w = (mpz_sizeinbase(md.v, 2) + 7) / 8;
  std::string out(w, '\0');
  to_bytes(r.v, reinterpret_cast<uint8_t*>(&out[0]), w);
  return py::bytes(out);
}

}  // namespace

PYBIND11_MODULE(_idc_paillier, m) {
  m.doc() = "Paillier encryption / homomorphic add / CRT decryption over GMP (secure-aggregation parity mode)";
  m.def("encrypt", &encrypt, py::arg("n"), py::arg("m"), py::arg("threads") = 8);
  m.def("add", &add, py::arg("n"), py::arg("a"), py::arg("b"));
  m.def("decrypt", &decrypt, py::arg("p"), py::arg("q"), py::arg("c"), py::arg("threads") = 8);
  m.def("powm", &powm, py::arg("base"), py::arg("exp"), py::arg("mod"));
}
