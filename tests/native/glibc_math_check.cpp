// Exhaustive / sampled comparison of csrc/glibc_math.h against the host libm.
// usage: glibc_math_check <func> [stride]   -> prints "<func> mismatches N of M"
// (the same header is what the GPU kernel runs; bit-exactness here means the
// kernel reproduces glibc's float libm results, i.e. the reference's).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "glibc_math.h"

static const gm::GmTables T = {GM_EXP2F_TAB, GM_LOGF_TAB, GM_POWF_TAB};

typedef float (*ff)(float);
static float g_expf(float x) { return gm::expf(x, T); }
static float g_exp2f(float x) { return gm::exp2f(x, T); }
static float g_logf(float x) { return gm::logf(x, T); }
static float g_tanhf(float x) { return gm::tanhf(x); }
static float g_atanf(float x) { return gm::atanf(x); }
static float g_expm1f(float x) { return gm::expm1f(x); }
static float g_log10f(float x) { return gm::log10f(x, T); }
static float g_acosf(float x) { return gm::acosf(x); }
// restricted-range functions: compare only inside the range the physics uses
static float g_cosf(float x) { return fabsf(x) < 120.0f ? gm::cosf(x) : ::cosf(x); }
static float g_tanf(float x) { return fabsf(x) < 120.0f ? gm::tanf(x) : ::tanf(x); }

struct Entry { const char* name; ff mine; ff ref; };
static const Entry FUNCS[] = {
    {"expf", g_expf, ::expf},
    {"exp2f", g_exp2f, ::exp2f},
    {"logf", g_logf, ::logf},
    {"tanhf", g_tanhf, ::tanhf},
    {"atanf", g_atanf, ::atanf},
    {"expm1f", g_expm1f, ::expm1f},
    {"log10f", g_log10f, ::log10f},
    {"acosf", g_acosf, ::acosf},
    {"cosf", g_cosf, ::cosf},
    {"tanf", g_tanf, ::tanf},
};

// powf: every x on a stride of the 2^32 patterns, for each y in a list
// (the exponents the reference uses + extras), plus a random (x, y) sweep.
static int check_powf(unsigned stride) {
  const float ys[] = {0.25f, -0.25f, 1.7f, 0.667f, 4.0f, 2.0f / 3.0f, 0.5f, 2.0f, 3.0f, -1.0f,
                      -0.5f, 1.5f, 0.2857143f, -0.0890f, -0.1222f, 11.5f, 7.25f, 5.08f,
                      -1.0f / 4.26f, -1.0f / 11.55f, 2.0f * 5.25f + 3.0f, 5.25f + 2.0f, 0.1f,
                      -3.0f, 10.0f, 1e-3f, -7.5f, 0.0f, 1.0f, 33.0f};
  unsigned long long bad = 0, n = 0;
  for (float y : ys) {
#pragma omp parallel for reduction(+ : bad, n) schedule(static, 65536)
    for (long long i = 0; i < (1LL << 32); i += stride) {
      const unsigned u = (unsigned)i;
      float x;
      memcpy(&x, &u, 4);
      const float a = gm::powf(x, y, T), b = ::powf(x, y);
      unsigned ua, ub;
      memcpy(&ua, &a, 4);
      memcpy(&ub, &b, 4);
      n++;
      if (!(ua == ub || (isnan(a) && isnan(b)))) {
        bad++;
#pragma omp critical
        if (bad < 2) fprintf(stderr, "powf(%a, %a): mine %a ref %a\n", x, y, a, b);
      }
    }
  }
#pragma omp parallel for reduction(+ : bad, n)
  for (long long i = 0; i < 400000000LL; ++i) {
    unsigned long long h = (unsigned long long)i * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    unsigned ux = (unsigned)h, uy = (unsigned)(h >> 32);
    uy = (uy & 0x80000000u) | (0x3c000000u + (uy & 0x07ffffffu));  // |y| in [2^-7, 2^8)
    float x, y;
    memcpy(&x, &ux, 4);
    memcpy(&y, &uy, 4);
    const float a = gm::powf(x, y, T), b = ::powf(x, y);
    unsigned ua, ub;
    memcpy(&ua, &a, 4);
    memcpy(&ub, &b, 4);
    n++;
    if (!(ua == ub || (isnan(a) && isnan(b)))) bad++;
  }
  printf("powf mismatches %llu of %llu\n", bad, n);
  return bad ? 1 : 0;
}

// powf_pair: every x on a stride, for pairs of exponents (wdfcnd's BEXP+2 and
// 2*BEXP+3 over the table's BEXP values, and special exponents), both results
// against host powf
static int check_powf_pair(unsigned stride) {
  const float bexps[] = {2.79f, 4.26f, 4.74f, 5.33f, 5.25f, 6.77f, 8.72f, 8.17f, 10.73f, 10.39f,
                         11.55f, 12.61f, 2.79f, 4.26f, 11.55f, 2.5f};
  const float extra[][2] = {{0.0f, 1.0f}, {1.0f, 0.0f}, {-2.0f, 3.0f}, {0.25f, -0.25f},
                            {INFINITY, 2.0f}, {2.0f, NAN}, {1e-3f, 33.0f}};
  unsigned long long bad = 0, n = 0;
  const int nb = sizeof(bexps) / sizeof(bexps[0]), ne = sizeof(extra) / sizeof(extra[0]);
  for (int j = 0; j < nb + ne; ++j) {
    const float y1 = j < nb ? bexps[j] + 2.0f : extra[j - nb][0];
    const float y2 = j < nb ? 2.0f * bexps[j] + 3.0f : extra[j - nb][1];
#pragma omp parallel for reduction(+ : bad, n) schedule(static, 65536)
    for (long long i = 0; i < (1LL << 32); i += stride) {
      const unsigned u = (unsigned)i;
      float x;
      memcpy(&x, &u, 4);
      float a1, a2;
      gm::powf_pair(x, y1, y2, T, a1, a2);
      const float b1 = ::powf(x, y1), b2 = ::powf(x, y2);
      unsigned ua1, ub1, ua2, ub2;
      memcpy(&ua1, &a1, 4);
      memcpy(&ub1, &b1, 4);
      memcpy(&ua2, &a2, 4);
      memcpy(&ub2, &b2, 4);
      n += 2;
      if (!(ua1 == ub1 || (isnan(a1) && isnan(b1)))) bad++;
      if (!(ua2 == ub2 || (isnan(a2) && isnan(b2)))) bad++;
    }
  }
  printf("powf_pair mismatches %llu of %llu\n", bad, n);
  return bad ? 1 : 0;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  if (!strcmp(argv[1], "powf")) return check_powf(argc > 2 ? (unsigned)atoi(argv[2]) : 3);
  if (!strcmp(argv[1], "powf_pair"))
    return check_powf_pair(argc > 2 ? (unsigned)atoi(argv[2]) : 3);
  const unsigned stride = argc > 2 ? (unsigned)atoi(argv[2]) : 1;
  for (const Entry& e : FUNCS) {
    if (strcmp(e.name, argv[1])) continue;
    unsigned long long bad = 0, n = 0;
    unsigned first = 0;
#pragma omp parallel for reduction(+ : bad, n) schedule(static, 65536)
    for (long long i = 0; i < (1LL << 32); i += stride) {
      const unsigned u = (unsigned)i;
      float x;
      memcpy(&x, &u, 4);
      const float a = e.mine(x), b = e.ref(x);
      unsigned ua, ub;
      memcpy(&ua, &a, 4);
      memcpy(&ub, &b, 4);
      const bool same = (ua == ub) || (isnan(a) && isnan(b));
      n++;
      if (!same) {
        bad++;
#pragma omp critical
        if (!first) {
          first = u ? u : 1;
          fprintf(stderr, "first mismatch x=%a (0x%08x): mine %a ref %a\n", x, u, a, b);
        }
      }
    }
    printf("%s mismatches %llu of %llu\n", e.name, bad, n);
    return bad ? 1 : 0;
  }
  fprintf(stderr, "unknown function %s\n", argv[1]);
  return 2;
}
