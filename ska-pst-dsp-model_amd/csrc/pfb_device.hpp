// pfb_device.hpp — CDNA4 (gfx950) device building blocks for the PFB kernels.
//
// * complex float32 helpers (float2, interleaved re/im like pfb_cf32)
// * register-resident small DFTs of any radix built from {2,3,4,5,7} by a
//   compile-time Cooley-Tukey split; twiddles are compile-time constants
//   computed in double (constexpr Taylor series) and rounded once to float
// * an LDS-resident mixed-radix Stockham pass that a whole workgroup applies to a
//   batch of rows; loads/stores of the first/last pass can be redirected to HBM
//   through functors so the FFT fuses with its producer/consumer.
//
// The transforms here are bandwidth-shaped (complex-float VALU butterflies, LDS
// exchange between passes); there is no dense contraction, so no MFMA.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include <utility>

namespace pfb {

// ------------------------------------------------------------------ complex helpers
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
// a * conj(b)
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, a.y * b.y), fmaf(a.y, b.x, -a.x * b.y));
}
// a * e^{DIR * i pi/2}: DIR=-1 -> -i*a, DIR=+1 -> +i*a
template <int DIR>
__device__ __forceinline__ float2 crot90(float2 a) {
  if constexpr (DIR < 0) return make_float2(a.y, -a.x);
  else return make_float2(-a.y, a.x);
}

// ------------------------------------------------------------------ constexpr trig
constexpr double kPi = 3.14159265358979323846264338327950288;

constexpr double taylor_sin(double x) {
  double term = x, sum = x;
  for (int i = 1; i < 24; ++i) {
    term *= -x * x / ((2.0 * i) * (2.0 * i + 1.0));
    sum += term;
  }
  return sum;
}
constexpr double taylor_cos(double x) {
  double term = 1.0, sum = 1.0;
  for (int i = 1; i < 24; ++i) {
    term *= -x * x / ((2.0 * i - 1.0) * (2.0 * i));
    sum += term;
  }
  return sum;
}
// cos/sin of 2 pi m / R, exact rational reduction into [-pi, pi]
constexpr double cos2pi(long m, long R) {
  m %= R;
  if (m < 0) m += R;
  if (2 * m > R) m -= R;
  return taylor_cos(2.0 * kPi * double(m) / double(R));
}
constexpr double sin2pi(long m, long R) {
  m %= R;
  if (m < 0) m += R;
  if (2 * m > R) m -= R;
  return taylor_sin(2.0 * kPi * double(m) / double(R));
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// generic complex helpers used by the small DFTs (overloaded for other complex types,
// e.g. the two-transform cpx2 of pfb_pair.hpp)
__device__ __forceinline__ float2 czero(float2) { return make_float2(0.f, 0.f); }
__device__ __forceinline__ float2 cneg(float2 a) { return make_float2(-a.x, -a.y); }
// c * a + b for real c
__device__ __forceinline__ float2 cfmar(float c, float2 a, float2 b) {
  return make_float2(fmaf(c, a.x, b.x), fmaf(c, a.y, b.y));
}
// a * (c + i s)
__device__ __forceinline__ float2 ctwc(float2 a, float c, float s) {
  return make_float2(fmaf(a.x, c, -a.y * s), fmaf(a.x, s, a.y * c));
}

// multiply by the compile-time twiddle e^{DIR * 2 pi i M / R}
template <int M, int R, int DIR, class C>
__device__ __forceinline__ C ctw(C a) {
  if constexpr ((M % R) == 0) {
    return a;
  } else if constexpr ((4 * M) % R == 0) {
    constexpr int q = ((4 * M) / R) % 4;  // multiples of pi/2
    if constexpr (q == 2) return cneg(a);
    else if constexpr (q == 1) return crot90<DIR>(a);
    else return crot90<-DIR>(a);
  } else {
    constexpr float c = (float)cos2pi(M, R);
    constexpr float s = (float)(DIR * sin2pi(M, R));
    return ctwc(a, c, s);
  }
}

// ------------------------------------------------------------------ small DFTs
constexpr int first_factor(int R) {
  if (R % 4 == 0 && R != 8) return 4;
  if (R % 2 == 0) return 2;
  if (R % 3 == 0) return 3;
  if (R % 5 == 0) return 5;
  if (R % 7 == 0) return 7;
  return R;
}

constexpr int cgcd(int a, int b) { return b == 0 ? a : cgcd(b, a % b); }
constexpr int ilog2(int n) { return n <= 1 ? 0 : 1 + ilog2(n / 2); }
// x^{-1} mod m (gcd(x, m) = 1)
constexpr int cinv_mod(int x, int m) {
  for (int i = 1; i < m; ++i)
    if ((x * i) % m == 1) return i;
  return m == 1 ? 0 : -1;
}

// In-place DFT of R points held in registers, natural order in and out.
// DIR = -1: X[k] = sum x[n] e^{-2 pi i n k / R}; DIR = +1: unnormalised inverse.
// C is float2 (one transform) or any complex type with the helpers above.
template <int R, int DIR, class C>
__device__ __forceinline__ void sdft(C* v) {
  if constexpr (R == 1) {
    return;
  } else if constexpr (R == 2) {
    C a = v[0];
    v[0] = cadd(a, v[1]);
    v[1] = csub(a, v[1]);
  } else if constexpr (R == 3) {
    constexpr float c = -0.5f;
    constexpr float s = (float)(DIR * 0.86602540378443864676372317075294);
    C t = cadd(v[1], v[2]);
    C d = csub(v[1], v[2]);
    C m = cfmar(c, t, v[0]);
    C ids = crot90<+1>(cscale(d, s));  // i s d
    v[0] = cadd(v[0], t);
    v[1] = cadd(m, ids);
    v[2] = csub(m, ids);
  } else if constexpr (R == 4) {
    C t0 = cadd(v[0], v[2]);
    C t1 = csub(v[0], v[2]);
    C t2 = cadd(v[1], v[3]);
    C t3 = crot90<DIR>(csub(v[1], v[3]));
    v[0] = cadd(t0, t2);
    v[2] = csub(t0, t2);
    v[1] = cadd(t1, t3);
    v[3] = csub(t1, t3);
  } else if constexpr (R == 5 || R == 7) {
    // direct symmetric form: pairs (n, R-n)
    constexpr int H = (R - 1) / 2;
    C sp[H], sm[H];
    static_for<0, H>([&](auto n) {
      sp[n] = cadd(v[n + 1], v[R - 1 - n]);
      sm[n] = csub(v[n + 1], v[R - 1 - n]);
    });
    C out[R];
    C x0 = v[0];
    C dc = x0;
    static_for<0, H>([&](auto n) { dc = cadd(dc, sp[n]); });
    out[0] = dc;
    static_for<1, H + 1>([&](auto k) {
      C re = x0;  // real-cos part
      C im = czero(x0);
      static_for<0, H>([&](auto n) {
        constexpr int nk = (decltype(n)::value + 1) * decltype(k)::value;
        constexpr float c = (float)cos2pi(nk, R);
        constexpr float s = (float)sin2pi(nk, R);
        re = cfmar(c, sp[n], re);
        im = cfmar(s, sm[n], im);
      });
      // X[k] = re + DIR * i * im ; X[R-k] = re - DIR * i * im
      C iim = crot90<+1>(im);  // i * im
      if constexpr (DIR < 0) {
        out[k] = csub(re, iim);
        out[R - k] = cadd(re, iim);
      } else {
        out[k] = cadd(re, iim);
        out[R - k] = csub(re, iim);
      }
    });
    static_for<0, R>([&](auto k) { v[k] = out[k]; });
  } else if constexpr (cgcd(first_factor(R), R / first_factor(R)) == 1) {
    // R = A B with A, B coprime (6, 12, 14, 28, ...): Good-Thomas prime-factor mapping, no
    // twiddles.  Input n = (B n1 + A n2) mod R; X[(B u k1 + A v k2) mod R] = z[k1][k2] with
    // u = B^{-1} mod A, v = A^{-1} mod B (W_R^{n k} = W_A^{n1 k1} W_B^{n2 k2}: the cross
    // terms are multiples of R).  Every index is a compile-time register permutation.
    constexpr int A = first_factor(R);
    constexpr int B = R / A;
    constexpr int U = cinv_mod(B % A, A), V = cinv_mod(A % B, B);
    static_assert(A > 1 && B > 1 && U > 0 && V > 0, "prime-factor split");
    C y[A][B];
    static_for<0, A>([&](auto n1) {
      static_for<0, B>([&](auto n2) {
        y[n1][n2] = v[(B * decltype(n1)::value + A * decltype(n2)::value) % R];
      });
      sdft<B, DIR>(y[n1]);
    });
    static_for<0, B>([&](auto k2) {
      C z[A];
      static_for<0, A>([&](auto n1) { z[n1] = y[n1][k2]; });
      sdft<A, DIR>(z);
      static_for<0, A>([&](auto k1) {
        v[(B * U * decltype(k1)::value + A * V * decltype(k2)::value) % R] = z[k1];
      });
    });
  } else {
    constexpr int A = first_factor(R);
    constexpr int B = R / A;
    static_assert(A * B == R && A > 1 && B > 1, "unsupported radix");
    C y[A][B];
    static_for<0, A>([&](auto n1) {
      static_for<0, B>([&](auto n2) { y[n1][n2] = v[A * n2 + n1]; });
      sdft<B, DIR>(y[n1]);
      static_for<1, B>([&](auto k1) {
        constexpr int m = decltype(n1)::value * decltype(k1)::value;
        y[n1][k1] = ctw<m, R, DIR>(y[n1][k1]);
      });
    });
    static_for<0, B>([&](auto k1) {
      C z[A];
      static_for<0, A>([&](auto n1) { z[n1] = y[n1][k1]; });
      sdft<A, DIR>(z);
      static_for<0, A>([&](auto k2) { v[k1 + B * k2] = z[k2]; });
    });
  }
}

// ------------------------------------------------------------------ LDS Stockham
// Padded LDS index: one spare float2 every 16 breaks the power-of-two strides of
// the radix-16 passes ("LDS layout").
__device__ __forceinline__ int lpad(int i) { return i + (i >> 4); }
__host__ __device__ constexpr int lds_row(int n) { return n + n / 16; }

// Radix lists of the compiled transform sizes.
template <int... Rs>
struct Radices {};

template <int N>
struct FFTPlan;
template <> struct FFTPlan<8> { using type = Radices<8>; };
template <> struct FFTPlan<16> { using type = Radices<16>; };
template <> struct FFTPlan<32> { using type = Radices<8, 4>; };
template <> struct FFTPlan<64> { using type = Radices<8, 8>; };
template <> struct FFTPlan<128> { using type = Radices<16, 8>; };
template <> struct FFTPlan<256> { using type = Radices<16, 16>; };
template <> struct FFTPlan<512> { using type = Radices<8, 8, 8>; };
template <> struct FFTPlan<1024> { using type = Radices<16, 16, 4>; };
template <> struct FFTPlan<2048> { using type = Radices<16, 16, 8>; };
template <> struct FFTPlan<4096> { using type = Radices<16, 16, 16>; };
// kept-bin widths W = Nf * de / nu of the synthesis
template <> struct FFTPlan<96> { using type = Radices<16, 6>; };
template <> struct FFTPlan<112> { using type = Radices<16, 7>; };
template <> struct FFTPlan<192> { using type = Radices<16, 12>; };
template <> struct FFTPlan<216> { using type = Radices<8, 27>; };
template <> struct FFTPlan<224> { using type = Radices<16, 14>; };
template <> struct FFTPlan<448> { using type = Radices<16, 28>; };
template <> struct FFTPlan<896> { using type = Radices<16, 8, 7>; };
// critically sampled channel counts (two-stage inversion, see mixed_chan_supported)
template <> struct FFTPlan<14> { using type = Radices<14>; };
template <> struct FFTPlan<28> { using type = Radices<4, 7>; };
template <> struct FFTPlan<56> { using type = Radices<8, 7>; };
template <> struct FFTPlan<432> { using type = Radices<16, 27>; };
template <> struct FFTPlan<864> { using type = Radices<16, 6, 9>; };
// ... and those channel counts times the combine factor (2 .. 16)
template <> struct FFTPlan<384> { using type = Radices<16, 24>; };
template <> struct FFTPlan<768> { using type = Radices<16, 16, 3>; };
template <> struct FFTPlan<1536> { using type = Radices<16, 16, 6>; };
template <> struct FFTPlan<1792> { using type = Radices<16, 16, 7>; };
template <> struct FFTPlan<3072> { using type = Radices<16, 16, 12>; };
template <> struct FFTPlan<3584> { using type = Radices<16, 16, 14>; };

// Default LDS accessors for a batch of rows stored at base + row * rs.
struct LdsIO {
  float2* base;
  int rs;
  __device__ __forceinline__ float2 load(int row, int i) const { return base[row * rs + lpad(i)]; }
  __device__ __forceinline__ void store(int row, int i, float2 v) const { base[row * rs + lpad(i)] = v; }
};

// LDS twiddle tables are padded by one slot every 32 entries: the power-of-two strided
// reads of twiddle_powers (index r m, m = k N / (NS R)) otherwise land on a few banks
// (e.g. m = 16 k: every even k on one bank).  Entry m sits at tw_slot(m); a table of n
// entries occupies tw_slots(n) float2 slots (even, so what follows stays 16-B aligned).
__host__ __device__ constexpr int tw_slot(int m) { return m + (m >> 5); }
__host__ __device__ constexpr int tw_slots(int n) { return (n + (n >> 5) + 2) & ~1; }

// Twiddle e^{DIR 2 pi i m / N} from a padded LDS table, entry m = e^{-2 pi i m / N}.
template <int DIR>
__device__ __forceinline__ float2 table_tw(const float2* __restrict__ tw, int m) {
  float2 w = tw[tw_slot(m)];
  if constexpr (DIR > 0) w.y = -w.y;
  return w;
}

// Twiddles w[r] = e^{DIR 2 pi i r m / N}, r = 1 .. R-1, from log2(R) table reads
// (r a power of two) and at most 3 complex products for the others (r = highest power of
// two below r, times the remainder): the reads issue back to back instead of R - 1
// dependent LDS round trips, at <= 3 roundings of error per twiddle.
__host__ __device__ constexpr int high_bit(int r) {
  int h = 1;
  while (2 * h <= r) h *= 2;
  return h;
}
template <int R, int DIR, class TW>
__device__ __forceinline__ void twiddle_powers(const TW& tw, int m, float2 (&w)[R]) {
  static_for<1, R>([&](auto rv) {
    constexpr int r = decltype(rv)::value;
    if constexpr (high_bit(r) == r) w[r] = table_tw<DIR>(tw, r * m);
  });
  static_for<1, R>([&](auto rv) {
    constexpr int r = decltype(rv)::value;
    constexpr int h = high_bit(r);
    if constexpr (h != r) w[r] = cmul(w[h], w[r - h]);
  });
}

// One Stockham autosort pass of radix R over `rows` transforms of length N held by
// the workgroup.  NS = product of the radices already applied.  Loads through `in`,
// stores through `out`.  All NT threads participate; the pass contains one barrier
// between its loads and its stores, so `in` and `out` may alias (in-place via
// registers).  The caller places a barrier before the next pass reads `out`.
struct LdsRows;
// WR (wave rows): every row's butterflies of every pass belong to one wave (wave_rows_ok), so
// an in-place pass over the LDS rows needs only a wave barrier (a wave's LDS instructions
// execute in order) — no workgroup barrier between its loads and stores
template <int N, int R, int NS, int DIR, int ROWS, int NT, bool WR = false, class In, class Out, class TW>
__device__ __forceinline__ void stockham_pass(const In& in, const Out& out, const TW& tw, int tid) {
  constexpr int NB = N / R;
  constexpr int TOT = ROWS * NB;
  constexpr int PER = (TOT + NT - 1) / NT;
  float2 v[PER][R];
  static_for<0, PER>([&](auto p) {
    const int b = tid + p * NT;
    if (TOT % NT == 0 || b < TOT) {
      const int row = b / NB, j = b - (b / NB) * NB;
      static_for<0, R>([&](auto r) { v[p][r] = in.load(row, j + r * NB); });
    }
  });
  if constexpr (In::kIsLds && Out::kIsLds) {
    if constexpr (WR && std::is_same_v<In, LdsRows> && std::is_same_v<Out, LdsRows>) __builtin_amdgcn_wave_barrier();
    else __syncthreads();
  }
  static_for<0, PER>([&](auto p) {
    const int b = tid + p * NT;
    if (TOT % NT == 0 || b < TOT) {
      const int row = b / NB, j = b - (b / NB) * NB;
      const int k = j % NS;
      if constexpr (NS > 1) {
        // e^{DIR 2 pi i r k / (NS R)} = table[(r k N / (NS R))]
        float2 w[R];
        twiddle_powers<R, DIR>(tw, k * (N / (NS * R)), w);
        static_for<1, R>([&](auto r) { v[p][r] = cmul(v[p][r], w[r]); });
      }
      sdft<R, DIR>(v[p]);
      const int idxD = (j / NS) * NS * R + k;
      static_for<0, R>([&](auto r) { out.store(row, idxD + r * NS, v[p][r]); });
    }
  });
}

// LDS row accessor (in-place passes need a barrier between loads and stores).
struct LdsRows : LdsIO {
  static constexpr bool kIsLds = true;
  __device__ LdsRows(float2* b, int r) : LdsIO{b, r} {}
};

// Run all passes of FFTPlan<N>; first pass loads via `first`, last pass stores via
// `last`, intermediate passes go through the LDS rows `lds`.  WR: see stockham_pass (the
// barrier between two passes is then a wave barrier too).
template <int N, int DIR, int ROWS, int NT, bool WR, int NS, int R, int... Rest, class First, class Last, class TW>
__device__ __forceinline__ void run_passes_impl(const First& first, const Last& last,
                                                const LdsRows& lds, const TW& tw, int tid) {
  if constexpr (sizeof...(Rest) == 0) {
    stockham_pass<N, R, NS, DIR, ROWS, NT, WR>(first, last, tw, tid);
  } else {
    stockham_pass<N, R, NS, DIR, ROWS, NT, WR>(first, lds, tw, tid);
    if constexpr (WR) __builtin_amdgcn_wave_barrier();
    else __syncthreads();
    run_passes_impl<N, DIR, ROWS, NT, WR, NS * R, Rest...>(lds, last, lds, tw, tid);
  }
}

template <int N, int DIR, int ROWS, int NT, bool WR = false, class First, class Last, int... Rs>
__device__ __forceinline__ void run_fft(const First& first, const Last& last, const LdsRows& lds,
                                        const float2* tw, int tid, Radices<Rs...>) {
  run_passes_impl<N, DIR, ROWS, NT, WR, 1, Rs...>(first, last, lds, tw, tid);
}

// Whether every pass of FFTPlan<N> over ROWS rows with NT threads gives each thread one
// butterfly (PER = 1) and keeps each row's butterflies inside one 64-lane wave: row = tid /
// (N / R) for every radix R, with N / R dividing 64.
template <int N, int ROWS, int NT, int... Rs>
constexpr bool wave_rows_ok_impl(Radices<Rs...>) {
  return ((ROWS * (N / Rs) == NT && 64 % (N / Rs) == 0) && ...);
}
template <int N, int ROWS, int NT>
constexpr bool wave_rows_ok() { return wave_rows_ok_impl<N, ROWS, NT>(typename FFTPlan<N>::type{}); }

// WR (round 6): wave-owned rows (wave_rows_ok), the passes ordered by wave barriers; the
// arithmetic is the same, so the output is bit-identical to the workgroup-barrier form
template <int N, int DIR, int ROWS, int NT, bool WR = false, class First, class Last>
__device__ __forceinline__ void block_fft(const First& first, const Last& last, const LdsRows& lds,
                                          const float2* tw, int tid) {
  static_assert(!WR || wave_rows_ok<N, ROWS, NT>(), "WR: a row's butterflies must stay in one wave");
  run_fft<N, DIR, ROWS, NT, WR>(first, last, lds, tw, tid, typename FFTPlan<N>::type{});
}


// Coordinates of the first pass of FFTPlan<N>.
template <int N, int ROWS, int NTH>
struct FirstPassOf {
  template <int R0, int... Rest>
  static constexpr int radix(Radices<R0, Rest...>) { return R0; }
  static constexpr int R = radix(typename FFTPlan<N>::type{});
  static constexpr int NB = N / R;
  static constexpr int TOT = ROWS * NB;
  static constexpr int PER = (TOT + NTH - 1) / NTH;
};

}  // namespace pfb
