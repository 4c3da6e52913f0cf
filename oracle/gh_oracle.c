/* gh_oracle.c — CPU restatement of Gen's particle-filter hot path.
 * TEST INFRASTRUCTURE ONLY (see gh_oracle.h for the scope statement and the
 * reference file:line map).  Plain C11, scalar, single thread.
 *
 * Build: oracle/Makefile (gcc -O2 -mfma -ffp-contract=off).  -ffp-contract=off
 * is required: every fused multiply-add in the specification
 * is written explicitly as fma(), every other product/sum is rounded
 * separately, exactly as in the HIP kernels.
 */
#include "gh_oracle.h"
#include "../gen_amd/csrc/gh_tables.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* The same source built with -fopenmp (liboracle_omp.so) runs the
   per-particle / per-chain loops on every host core: used only for the
   all-cores CPU baseline of bench.py.  Every parallel loop computes values
   that depend on its own index alone; reductions stay serial in index order,
   so both builds give identical results. */
int orc_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ------------------------------------------------------------------ bits */
static double f64_of(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static uint64_t u64_of(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

/* ----------------------------------------------------------- Philox4x32 */
static uint32_t mulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint32_t h0 = mulhi(0xD2511F53u, c0), l0 = 0xD2511F53u * c0;
    uint32_t h1 = mulhi(0xCD9E8D57u, c2), l1 = 0xCD9E8D57u * c2;
    uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
    c0 = n0; c1 = l1; c2 = n2; c3 = l0;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

enum { S_INIT = 1, S_STEP = 2, S_RESAMPLE = 3, S_SAMPLE = 4, S_IS = 5, S_MH = 6, S_SIM = 7 };
enum { SIM_OBS_DRAW = 32 };

static void rng(uint64_t seed, uint64_t id, uint32_t step, uint32_t stream, uint32_t draw,
                uint32_t out[4]) {
  uint32_t c[4] = {(uint32_t)id, (uint32_t)(id >> 32), step, (stream << 16) | draw};
  uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  orc_philox4x32_10(c, k, out);
}
static uint64_t bits53(uint32_t a, uint32_t b) { return ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6); }
static double unif53(uint32_t a, uint32_t b) { return (double)bits53(a, b) * 0x1p-53; }

/* ------------------------------------------------------------------ exp */
static double scale2k(double p, int k) {
  if (k > -1022 && k < 1024) return p * f64_of((uint64_t)(k + 1023) << 52);
  if (k >= 1024) return (p * 0x1p1023) * 2.0;
  return (p * f64_of((uint64_t)(k + 600 + 1023) << 52)) * 0x1p-600;
}

double orc_exp(double x) {
  if (x != x) return x;
  if (x < -745.5) return 0.0;
  if (x > 709.78) return INFINITY;
  double k = rint(x * 0x1.71547652b82fep+0);
  double r = fma(-k, 0x1.62e42fee00000p-1, x);
  r = fma(-k, 0x1.a39ef35793c76p-33, r);
  static const double c[14] = {
      1.0, 1.0, 0x1.0000000000000p-1, 0x1.5555555555555p-3, 0x1.5555555555555p-5,
      0x1.1111111111111p-7, 0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-13, 0x1.a01a01a01a01ap-16,
      0x1.71de3a556c734p-19, 0x1.27e4fb7789f5cp-22, 0x1.ae64567f544e4p-26, 0x1.1eed8eff8d898p-29,
      0x1.6124613a86d09p-33};
  double p = c[13];
  for (int n = 12; n >= 0; --n) p = fma(p, r, c[n]);
  return scale2k(p, (int)k);
}

/* ------------------------------------------------------------------ log */
double orc_log(double x) {
  if (x != x || x < 0.0) return NAN;
  if (x == 0.0) return -INFINITY;
  if (x == INFINITY) return x;
  int k = 0;
  uint64_t b = u64_of(x);
  if (b < 0x0010000000000000ull) { x *= 0x1p54; k = -54; b = u64_of(x); }
  k += (int)(b >> 52) - 1023;
  double m = f64_of((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
  if (m > 0x1.6a09e667f3bcdp+0) { m *= 0.5; k += 1; }
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  double f = m - 1.0;
  double s = f / (2.0 + f);
  double z = s * s, w = z * z;
  double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  double R = t2 + t1;
  double hfsq = 0.5 * f * f;
  double dk = (double)k;
  return dk * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + dk * 1.90821492927058770002e-10)) - f);
}

/* -------------------------------------------------------------- sin/cos */
static double ksin(double x) {
  static const double c[7] = {-0x1.5555555555555p-3, 0x1.1111111111111p-7, -0x1.a01a01a01a01ap-13,
                              0x1.71de3a556c734p-19, -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33,
                              -0x1.ae7f3e733b81fp-41};
  double x2 = x * x, p = c[6];
  for (int n = 5; n >= 0; --n) p = fma(p, x2, c[n]);
  return fma(x * x2, p, x);
}
static double kcos(double x) {
  static const double c[8] = {-0x1.0000000000000p-1, 0x1.5555555555555p-5, -0x1.6c16c16c16c17p-10,
                              0x1.a01a01a01a01ap-16, -0x1.27e4fb7789f5cp-22, 0x1.1eed8eff8d898p-29,
                              -0x1.93974a8c07c9dp-37, 0x1.ae7f3e733b81fp-45};
  double x2 = x * x, p = c[7];
  for (int n = 6; n >= 0; --n) p = fma(p, x2, c[n]);
  return fma(x2, p, 1.0);
}

void orc_sincos_2pi(double u, double* s, double* c) {
  double v = u * 8.0, o = floor(v), f = v - o;
  int oi = (int)o;
  double ss, cc;
  if (oi & 1) { double b = (1.0 - f) * 0x1.921fb54442d18p-1; ss = kcos(b); cc = ksin(b); }
  else { double a = f * 0x1.921fb54442d18p-1; ss = ksin(a); cc = kcos(a); }
  switch (oi >> 1) {
    case 0: *s = ss; *c = cc; break;
    case 1: *s = cc; *c = -ss; break;
    case 2: *s = -ss; *c = -cc; break;
    default: *s = -cc; *c = ss; break;
  }
}

double orc_cos(double x) {
  double k = rint(x * 0x1.45f306dc9c883p-1);
  double r = fma(-k, 1.57079632673412561417e+00, x);
  r = fma(-k, 6.07710050630396597660e-11, r);
  r = fma(-k, 2.02226624871116645580e-21, r);
  switch (((int)k) & 3) {
    case 0: return kcos(r);
    case 1: return -ksin(r);
    case 2: return -kcos(r);
    default: return ksin(r);
  }
}

/* sin/cos(2 pi c 2^-32) of a 32-bit angle word, table driven:
   nearest of 256 table angles j = (c + 2^23) >> 24 mod 256, residual
   d = (int32)(c - j 2^24) * (2 pi 2^-32), short Taylor polynomials of sin d and
   cos d - 1, rotation by the table's {sin, cos}(2 pi j / 256).  The table data
   is gen_amd/csrc/gh_tables.h (tools/gen_tables.py). */
static const double math_tab[768] = {GH_LOG_TABLE_DATA, GH_TRIG_TABLE_DATA};

void orc_sincos_2pi_u32(uint32_t c, double* s, double* co) {
  const double* t = math_tab + 256;
  uint32_t j = ((c + 0x800000u) >> 24) & 255u;
  int32_t di = (int32_t)(c - (j << 24));
  double d = (double)di * 0x1.921fb54442d18p-30;
  double d2 = d * d;
  double ps = fma(d2, -0x1.a01a01a01a01ap-13, 0x1.1111111111111p-7);
  ps = fma(d2, ps, -0x1.5555555555555p-3);
  double sd = fma(d * d2, ps, d);
  double pc = fma(d2, -0x1.6c16c16c16c17p-10, 0x1.5555555555555p-5);
  pc = fma(d2, pc, -0.5);
  double cm1 = d2 * pc;
  double sj = t[2 * j], cj = t[2 * j + 1];
  *s = sj + fma(sj, cm1, cj * sd);
  *co = cj + fma(cj, cm1, -(sj * sd));
}

/* Table-driven log of x in [2^-53, 1] (the table is the shared
   data of gen_amd/csrc/gh_tables.h, made by tools/gen_tables.py):
   log x = k ln2 + logc_i + log1p(r), r = fma(m, invc_i, -1),
   log1p(r) = r + r^2 (-1/2 + r/3 - r^2/4 + r^3/5 - r^4/6 + r^5/7). */
static const double* log_tab = math_tab;
double orc_log_unit(double x) {
  uint64_t b = u64_of(x);
  uint32_t i = (uint32_t)(b >> 45) & 127u;
  int up = i >= 53;
  int k = (int)(b >> 52) - 1023 + up;
  double m = f64_of((b & 0x000FFFFFFFFFFFFFull) | ((uint64_t)(1023 - up) << 52));
  double r = fma(m, log_tab[2 * i], -1.0);
  double r2 = r * r;
  double q = fma(0x1.2492492492492p-3, r, -0x1.5555555555555p-3);
  q = fma(q, r, 0x1.999999999999ap-3);
  q = fma(q, r, -0x1.0p-2);
  q = fma(q, r, 0x1.5555555555555p-2);
  q = fma(q, r, -0x1.0p-1);
  double kd = (double)k;
  double h = fma(kd, 0x1.62e42fefa3800p-1, log_tab[2 * i + 1]);
  double l = fma(kd, 0x1.ef35793c76730p-45, r);
  return h + fma(r2, q, l);
}

/* Box–Muller on three words: radius from 1 - u53(a, b) (exact), angle word c */
static void box_muller(uint32_t a, uint32_t b, uint32_t c, double* z0, double* z1) {
  uint32_t hi = a >> 11, lo = ((a << 21) & 0xFC000000u) | (b >> 6);
  double u1 = fma(-(double)lo, 0x1p-53, fma(-(double)hi, 0x1p-21, 1.0)); /* = 1 - u53(a, b) */
  double r = sqrt(-2.0 * orc_log_unit(u1));
  double s, co;
  orc_sincos_2pi_u32(c, &s, &co);
  *z0 = r * co;
  *z1 = r * s;
}

void orc_box_muller(uint32_t a, uint32_t b, uint32_t c, double* z0, double* z1) { box_muller(a, b, c, z0, z1); }

/* n standard normals for (id, step, stream) from blocks base, base+1, ...:
   pair p takes words 3p, 3p+1, 3p+2 of the concatenated blocks */
static void normals_at(uint64_t seed, uint64_t id, uint32_t step, uint32_t stream, uint32_t base, int n,
                       double* z) {
  uint32_t w[4];
  int cur = -1;
  for (int p = 0; 2 * p < n; ++p) {
    uint32_t wd[3];
    for (int q = 0; q < 3; ++q) {
      int k = 3 * p + q;
      if ((k >> 2) != cur) { cur = k >> 2; rng(seed, id, step, stream, base + (uint32_t)cur, w); }
      wd[q] = w[k & 3];
    }
    double a, c;
    box_muller(wd[0], wd[1], wd[2], &a, &c);
    z[2 * p] = a;
    if (2 * p + 1 < n) z[2 * p + 1] = c;
  }
}
void orc_normals(uint64_t seed, uint64_t id, uint32_t step, uint32_t stream, int n, double* z) {
  normals_at(seed, id, step, stream, 0, n, z);
}

static uint64_t scale_u53(uint64_t u, uint64_t S) {
  unsigned __int128 p = (unsigned __int128)u * S;
  return (uint64_t)(p >> 53);
}
static int qshift(uint64_t n) {
  int lg = 0;
  while ((1ull << lg) < n) ++lg;
  int s = 62 - lg;
  return s > 52 ? 52 : s;
}
static uint64_t quantize(double lw, double M, int shift) {
  double e = orc_exp(lw - M);
  return (uint64_t)(e * f64_of((uint64_t)(shift + 1023) << 52));
}

double orc_normal_logpdf(double x, double mu, double std) {
  /* normal.jl:56-60, literally */
  double var = std * std;
  double diff = x - mu;
  return -(diff * diff) / (2.0 * var) - 0.5 * orc_log(2.0 * 0x1.921fb54442d18p+1 * var);
}

/* ------------------------------------------------------- linear algebra */
/* Cholesky–Banachiewicz, row-major, lower factor in L (full d*d storage). */
static int chol(int d, const double* S, double* L) {
  memset(L, 0, sizeof(double) * d * d);
  for (int i = 0; i < d; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = S[i * d + j];
      for (int k = 0; k < j; ++k) s = fma(-L[i * d + k], L[j * d + k], s);
      if (i == j) {
        if (!(s > 0.0)) return -1;
        L[i * d + i] = sqrt(s);
      } else {
        L[i * d + j] = s / L[j * d + j];
      }
    }
  return 0;
}
/* Y = L^{-1} B for B (d x m) row-major */
static void fwdsub(int d, int m, const double* L, const double* B, double* Y) {
  for (int c = 0; c < m; ++c)
    for (int i = 0; i < d; ++i) {
      double s = B[i * m + c];
      for (int k = 0; k < i; ++k) s = fma(-L[i * d + k], Y[k * m + c], s);
      Y[i * m + c] = s / L[i * d + i];
    }
}
/* X = L^{-T} B for B (d x m) row-major */
static void bwdsub(int d, int m, const double* L, const double* B, double* X) {
  for (int c = 0; c < m; ++c)
    for (int i = d - 1; i >= 0; --i) {
      double s = B[i * m + c];
      for (int k = i + 1; k < d; ++k) s = fma(-L[k * d + i], X[k * m + c], s);
      X[i * m + c] = s / L[i * d + i];
    }
}
/* C = A B (n x k times k x m), fma over the inner index ascending */
static void matmul(int n, int k, int m, const double* A, const double* B, double* C) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < m; ++j) {
      double acc = 0.0;
      for (int l = 0; l < k; ++l) acc = fma(A[i * k + l], B[l * m + j], acc);
      C[i * m + j] = acc;
    }
}
static double gauss_cst(int d, const double* L) {
  double acc = 0.0;
  for (int i = 0; i < d; ++i) acc += orc_log(L[i * d + i]);
  double logdet = 2.0 * acc;
  return -0.5 * ((double)d * 0x1.d67f1c864beb4p+0 + logdet);
}

/* ----------------------------------------------------------- the models */
typedef struct {
  int family, d, dy, k, v;
  /* LGSSM */
  double *A, *b, *LQ, *M, *LR, *c, *mu0, *L0, cstR, cstQ, cst0;
  int lq_diag, m_diag;  /* exact-zero structure: skipped terms */
  /* locally optimal proposal p(x_t | x_{t-1}, y_t): S = H Q H^T + R,
     K^T = S^{-1} H Q, F = I - K H, Sigma = F Q; at t = 1 the same with P0 */
  int opt;
  double *H, *LS, *Kt, *FA, *Fb, *LSig, *WA, *Wb, *LS1, *Kt1, *LSig1, cstS, cstS1;
  /* HMM */
  double *prior, *T, *E, *logE;
  /* Kitagawa; the prior densities for the Gaussian custom proposal's weight,
     and that proposal's arguments (alpha, beta, gamma, sigma_q) with
     1/(2 sigma_q^2), -0.5 log(2 pi sigma_q^2) */
  double mu1, s1, sx, sy, inv2vy, csty, inv2vx, cstx, inv2v1, cst1;
  double qa[6];
  /* LGSSM, the user-parameterised linear-Gaussian proposal N(P x_{t-1} + u, Sigma_q):
     P, chol(Sigma_q), its log-normaliser, the next steps' u (orc_pf_set_proposal_args) */
  int qlin;
  double *QP, *QL, cstq, qu[64];
  /* regression (quickstart.jl:3-9): priors, 1/(2 sigma^2), -0.5 log(2 pi sigma^2), xs */
  double mu_s, sd_s, mu_i, sd_i, sigma, inv2v, cst, inv2s, csts, inv2i, csti;
  double xs[32];
  /* slot family (gen_amd/csrc/gh_slots.h): latent form, slot count, each slot's
     distribution, value count, mean form, offsets in obs_t.bt and in the
     observation vector, parameter block (mvnormal M = L_R^-1 H | H | c | L_R;
     normal / poisson / bernoulli h | c; categorical W | c) and constants */
  int lat, K, sdist[4], sm[4], slink[4], svoff[4], syoff[4], snv, uin;  /* uin: per-step latent inputs (form 2) */
  /* switching latent (form 4): nz regimes, state x[dx] | one-hot z[nz]; prior, T as
     the categorical latent's; SW: per regime A_z | b_z | chol(Q_z); mu0, L0 */
  int nz;
  double* SW;
  double cstQz[8];
  /* dependencies between a step's observed addresses: slot k's linear predictor
     adds the fma chain of sdg[k][j] y_j over its parents j < k (sdep: slots with parents) */
  int sdep;
  double sdg[4][4];
  double* sP[4];
  double scst[4], sinv2v[4], ssd[4];
} model_t;

static void model_free(model_t* m) {
  free(m->QP); free(m->QL);
  free(m->A); free(m->b); free(m->LQ); free(m->M); free(m->LR); free(m->c); free(m->mu0);
  free(m->L0); free(m->prior); free(m->T); free(m->E); free(m->logE);
  free(m->H); free(m->LS); free(m->Kt); free(m->FA); free(m->Fb); free(m->LSig); free(m->WA); free(m->Wb);
  free(m->LS1); free(m->Kt1); free(m->LSig1);
  for (int k = 0; k < 4; ++k) free(m->sP[k]);
  free(m->SW);
}

/* the optimal proposal's factors for state prior covariance P: chol(S), K^T,
   chol(Sigma) and (optionally) F; returns 0 when S and Sigma are positive definite */
static int opt_derive(int d, int dy, const double* H, const double* R, const double* P, double* LS, double* Kt,
                      double* LSig, double* F_out) {
  double* HP = malloc(sizeof(double) * dy * d);
  double* S = malloc(sizeof(double) * dy * dy);
  double* Y = malloc(sizeof(double) * dy * d);
  double* F = malloc(sizeof(double) * d * d);
  double* Sig = malloc(sizeof(double) * d * d);
  int rc = 0;
  matmul(dy, d, d, H, P, HP);
  for (int r = 0; r < dy; ++r)
    for (int q = 0; q < dy; ++q) {
      double acc = R[r * dy + q];
      for (int j = 0; j < d; ++j) acc = fma(HP[r * d + j], H[q * d + j], acc);
      S[r * dy + q] = acc;
    }
  if (chol(dy, S, LS)) { rc = -1; goto out; }
  fwdsub(dy, d, LS, HP, Y);
  bwdsub(dy, d, LS, Y, Kt);
  for (int i = 0; i < d; ++i)
    for (int j = 0; j < d; ++j) {
      double acc = i == j ? 1.0 : 0.0;
      for (int r = 0; r < dy; ++r) acc = fma(-Kt[r * d + i], H[r * d + j], acc);
      F[i * d + j] = acc;
    }
  matmul(d, d, d, F, P, Sig);
  if (chol(d, Sig, LSig)) { rc = -1; goto out; }
  if (F_out) memcpy(F_out, F, sizeof(double) * d * d);
out:
  free(HP); free(S); free(Y); free(F); free(Sig);
  return rc;
}

/* a library slot (dist 6, m = the distribution id of gh_dists.h): the scalar
   distributions and their argument counts (lib_nargs); argument j is
   link_j(c_j + h_j.x), link 0 identity, 2 exp, 3 logistic */
static int slot_lib_nargs(int dist) {
  switch (dist) {
    case 6: case 11: case 12: case 15: return 1;
    case 1: case 4: case 5: case 8: case 9: case 10: case 13: case 14: case 16: case 17: return 2;
    case 19: return 3;
    default: return 0;
  }
}
static int model_build(model_t* m, int family, int d, int dy, int k, int v, const double* p,
                       int64_t np) {
  memset(m, 0, sizeof(*m));
  m->family = family; m->d = d; m->dy = dy; m->k = k; m->v = v;
  if (family == ORC_LGSSM) {
    int64_t need = (int64_t)d * d + d + (int64_t)d * d + (int64_t)dy * d + dy + (int64_t)dy * dy + d + (int64_t)d * d;
    if (np < need) return -1;
    const double *A = p, *b = A + d * d, *Q = b + d, *H = Q + d * d, *c = H + dy * d, *R = c + dy,
                 *mu0 = R + dy * dy, *P0 = mu0 + d;
    m->A = malloc(sizeof(double) * d * d); memcpy(m->A, A, sizeof(double) * d * d);
    m->b = malloc(sizeof(double) * d); memcpy(m->b, b, sizeof(double) * d);
    m->LQ = malloc(sizeof(double) * d * d);
    if (chol(d, Q, m->LQ)) return -2;
    m->LR = malloc(sizeof(double) * dy * dy);
    if (chol(dy, R, m->LR)) return -2;
    m->M = malloc(sizeof(double) * dy * d);
    fwdsub(dy, d, m->LR, H, m->M);
    m->c = malloc(sizeof(double) * dy); memcpy(m->c, c, sizeof(double) * dy);
    m->mu0 = malloc(sizeof(double) * d); memcpy(m->mu0, mu0, sizeof(double) * d);
    m->L0 = malloc(sizeof(double) * d * d);
    if (chol(d, P0, m->L0)) return -2;
    m->cstR = gauss_cst(dy, m->LR);
    m->cstQ = gauss_cst(d, m->LQ);
    m->cst0 = gauss_cst(d, m->L0);
    m->lq_diag = 1;
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < i; ++j) if (m->LQ[i * d + j] != 0.0) m->lq_diag = 0;
    m->m_diag = dy == d;
    for (int r = 0; m->m_diag && r < dy; ++r)
      for (int j = 0; j < d; ++j) if (j != r && m->M[r * d + j] != 0.0) m->m_diag = 0;
    /* locally optimal proposal (engine: gh_model_create; needs d + dy <= 32) */
    m->H = malloc(sizeof(double) * dy * d); memcpy(m->H, H, sizeof(double) * dy * d);
    m->LS = calloc(dy * dy, sizeof(double)); m->Kt = calloc(dy * d, sizeof(double));
    m->LSig = calloc(d * d, sizeof(double)); m->LS1 = calloc(dy * dy, sizeof(double));
    m->Kt1 = calloc(dy * d, sizeof(double)); m->LSig1 = calloc(d * d, sizeof(double));
    m->FA = calloc(d * d, sizeof(double)); m->Fb = calloc(d, sizeof(double));
    m->WA = calloc(dy * d, sizeof(double)); m->Wb = calloc(dy, sizeof(double));
    double* F = malloc(sizeof(double) * d * d);
    m->opt = d + dy <= 32 && opt_derive(d, dy, H, R, Q, m->LS, m->Kt, m->LSig, F) == 0 &&
             opt_derive(d, dy, H, R, P0, m->LS1, m->Kt1, m->LSig1, NULL) == 0;
    if (m->opt) {
      matmul(d, d, d, F, A, m->FA);
      matmul(d, d, 1, F, b, m->Fb);
      double* W = malloc(sizeof(double) * dy * d);
      fwdsub(dy, d, m->LS, H, W);
      matmul(dy, d, d, W, A, m->WA);
      matmul(dy, d, 1, W, b, m->Wb);
      free(W);
      m->cstS = gauss_cst(dy, m->LS);
      m->cstS1 = gauss_cst(dy, m->LS1);
    }
    free(F);
  } else if (family == ORC_HMM) {
    if (np < (int64_t)k + (int64_t)k * k + (int64_t)v * k) return -1;
    m->d = 1;
    m->prior = malloc(sizeof(double) * k); memcpy(m->prior, p, sizeof(double) * k);
    m->T = malloc(sizeof(double) * k * k); memcpy(m->T, p + k, sizeof(double) * k * k);
    m->E = malloc(sizeof(double) * v * k); memcpy(m->E, p + k + k * k, sizeof(double) * v * k);
    m->logE = malloc(sizeof(double) * v * k);
    for (int i = 0; i < v * k; ++i) m->logE[i] = orc_log(m->E[i]);
  } else if (family == ORC_KITAGAWA) {
    if (np < 4) return -1;
    m->d = 1;
    m->mu1 = p[0]; m->s1 = p[1];
    m->sx = sqrt(p[2]);
    m->sy = sqrt(p[3]);
    m->inv2vy = 1.0 / (2.0 * p[3]);
    m->csty = -0.5 * orc_log(2.0 * 0x1.921fb54442d18p+1 * p[3]);
    m->inv2vx = 1.0 / (2.0 * p[2]);
    m->cstx = -0.5 * orc_log(2.0 * 0x1.921fb54442d18p+1 * p[2]);
    m->inv2v1 = 1.0 / (2.0 * (p[1] * p[1]));
    m->cst1 = -0.5 * orc_log(2.0 * 0x1.921fb54442d18p+1 * (p[1] * p[1]));
  } else if (family == ORC_SLOTS) {
    /* include/gen_hip.h GH_FAMILY_SLOTS (the engine's slots_build, same checks) */
    if (d < 1 || d > 16 || np < 2) return -1;
    m->lat = (int)p[0]; m->K = (int)p[1];
    if ((double)m->lat != p[0] || m->lat < 0 || m->lat > 4 || (m->lat == 1 && d != 1) || (m->lat == 3 && d < 2))
      return -1;
    m->uin = m->lat == 2;  /* affine with per-step inputs: x_t ~ mvnormal(A x + (b + u_t), Q) */
    if (m->uin) m->lat = 0;
    if ((double)m->K != p[1] || m->K < 1 || m->K > 4) return -1;
    int64_t i = 2 + 3 * (int64_t)m->K;
    if (np < i) return -1;
    int voff = 0, yoff = 0;
    for (int k = 0; k < m->K; ++k) {
      const double* hd = p + 2 + 3 * k;
      int dist = (int)hd[0], mm = (int)hd[1], link = (int)hd[2], nv = 1;
      if ((double)dist != hd[0] || (double)mm != hd[1] || (double)link != hd[2]) return -1;
      if (dist == 1) { if (link != 0 || mm < 1 || mm > 32) return -1; nv = mm; }
      else if (dist == 2) { if (mm != 1 || !(link == 0 || link == 5 || (link == 1 && d == 1))) return -1; }
      else if (dist == 3) { if (mm != 1 || link != 2) return -1; nv = 2; }
      else if (dist == 4) { if (mm != 1 || link != 3) return -1; }
      else if (dist == 5) { if (mm < 2 || mm > 16 || link != 4) return -1; }
      else if (dist == 6) { if (slot_lib_nargs(mm) == 0 || link != 0) return -1; }
      else return -1;
      m->sdist[k] = dist; m->sm[k] = mm; m->slink[k] = link;
      m->svoff[k] = voff; m->syoff[k] = yoff;
      voff += nv; yoff += dist == 1 ? mm : 1;
    }
    if (voff + (m->uin ? d : 0) > 32 || yoff > 32) return -1;
    m->dy = yoff;
    m->snv = voff;  /* (the input, then the linear proposal's u_t, follow these values on the device) */
    if (m->lat == 0) {
      int64_t need = 3 * (int64_t)d * d + 2 * (int64_t)d;
      if (np < i + need) return -1;
      const double *A = p + i, *b = A + d * d, *Q = b + d, *mu0 = Q + d * d, *P0 = mu0 + d;
      m->A = malloc(sizeof(double) * d * d); memcpy(m->A, A, sizeof(double) * d * d);
      m->b = malloc(sizeof(double) * d); memcpy(m->b, b, sizeof(double) * d);
      m->LQ = malloc(sizeof(double) * d * d);
      if (chol(d, Q, m->LQ)) return -2;
      m->mu0 = malloc(sizeof(double) * d); memcpy(m->mu0, mu0, sizeof(double) * d);
      m->L0 = malloc(sizeof(double) * d * d);
      if (chol(d, P0, m->L0)) return -2;
      m->cstQ = gauss_cst(d, m->LQ);
      m->cst0 = gauss_cst(d, m->L0);
      i += need;
    } else if (m->lat == 4) {  /* switching: nz prior[nz] T[nz*nz] (A_z b_z Q_z per regime) mu0 P0 */
      if (np < i + 1) return -1;
      int nz = (int)p[i], dx = d - nz;
      if ((double)nz != p[i] || nz < 2 || nz > 8 || dx < 1) return -1;
      int64_t per = 2 * (int64_t)dx * dx + dx;
      int64_t need = 1 + nz + (int64_t)nz * nz + nz * per + dx + (int64_t)dx * dx;
      if (np < i + need) return -1;
      const double* pr = p + i + 1;
      for (int64_t j = 0; j < nz + (int64_t)nz * nz; ++j)
        if (!(pr[j] >= 0.0) || pr[j] == INFINITY) return -1;
      m->nz = nz;
      m->prior = malloc(sizeof(double) * nz); memcpy(m->prior, pr, sizeof(double) * nz);
      m->T = malloc(sizeof(double) * nz * nz); memcpy(m->T, pr + nz, sizeof(double) * nz * nz);
      m->SW = malloc(sizeof(double) * (size_t)(nz * per));
      const double* rb = pr + nz + nz * nz;
      for (int z = 0; z < nz; ++z, rb += per) {
        double* blk = m->SW + z * per;
        memcpy(blk, rb, sizeof(double) * (size_t)(dx * dx + dx));
        if (chol(dx, rb + dx * dx + dx, blk + dx * dx + dx)) return -2;
        m->cstQz[z] = gauss_cst(dx, blk + dx * dx + dx);
      }
      m->mu0 = malloc(sizeof(double) * dx); memcpy(m->mu0, rb, sizeof(double) * dx);
      m->L0 = malloc(sizeof(double) * dx * dx);
      if (chol(dx, rb + dx, m->L0)) return -2;
      m->cst0 = gauss_cst(dx, m->L0);
      i += need;
    } else if (m->lat == 3) {  /* categorical latent: prior[K] T[K*K] (T[new*K + prev]), one-hot state */
      int64_t need = (int64_t)d + (int64_t)d * d;
      if (np < i + need) return -1;
      for (int64_t j = 0; j < need; ++j)
        if (!(p[i + j] >= 0.0) || p[i + j] == INFINITY) return -1;
      m->prior = malloc(sizeof(double) * d); memcpy(m->prior, p + i, sizeof(double) * d);
      m->T = malloc(sizeof(double) * d * d); memcpy(m->T, p + i + d, sizeof(double) * d * d);
      i += need;
    } else {
      if (np < i + 3 || !(p[i + 1] > 0.0) || !(p[i + 2] > 0.0)) return -1;
      double s1 = p[i + 1], sdx = p[i + 2];
      m->mu1 = p[i]; m->s1 = s1; m->sx = sdx;  /* normal.jl:56-60: var = sd * sd */
      m->inv2vx = 1.0 / (2.0 * (sdx * sdx));
      m->cstx = -0.5 * orc_log(2.0 * 0x1.921fb54442d18p+1 * (sdx * sdx));
      m->inv2v1 = 1.0 / (2.0 * (s1 * s1));
      m->cst1 = -0.5 * orc_log(2.0 * 0x1.921fb54442d18p+1 * (s1 * s1));
      i += 3;
    }
    for (int k = 0; k < m->K; ++k) {
      int mm = m->sm[k];
      if (m->sdist[k] == 1) {
        int64_t need = (int64_t)mm * d + mm + (int64_t)mm * mm;
        if (np < i + need) return -1;
        const double *H = p + i, *c = H + mm * d, *R = c + mm;
        double* blk = calloc((size_t)(2 * mm * d + mm + mm * mm), sizeof(double));
        m->sP[k] = blk;
        double* LR = blk + 2 * mm * d + mm;
        if (chol(mm, R, LR)) return -2;
        fwdsub(mm, d, LR, H, blk);
        memcpy(blk + mm * d, H, sizeof(double) * mm * d);
        memcpy(blk + 2 * mm * d, c, sizeof(double) * mm);
        m->scst[k] = gauss_cst(mm, LR);
        i += need;
      } else if (m->sdist[k] == 2 && m->slink[k] == 5) {  /* h c g s: sd = exp(g.x + s) */
        int64_t need = 2 * (int64_t)d + 2;
        if (np < i + need) return -1;
        m->sP[k] = malloc(sizeof(double) * need);
        memcpy(m->sP[k], p + i, sizeof(double) * need);
        i += need;
      } else if (m->sdist[k] == 2) {
        int64_t need = m->slink[k] == 0 ? d + 2 : 1;
        if (np < i + need) return -1;
        m->sP[k] = calloc((size_t)d + 1, sizeof(double));
        if (m->slink[k] == 0) memcpy(m->sP[k], p + i, sizeof(double) * (d + 1));
        double sd = p[i + need - 1];
        if (!(sd > 0.0)) return -1;
        m->ssd[k] = sd;
        m->sinv2v[k] = 1.0 / (2.0 * (sd * sd));
        m->scst[k] = -0.5 * orc_log(2.0 * 0x1.921fb54442d18p+1 * (sd * sd));
        i += need;
      } else if (m->sdist[k] == 6) {  /* (link h[d] c) per argument */
        int na = slot_lib_nargs(mm);
        int64_t need = (int64_t)na * (d + 2);
        if (np < i + need) return -1;
        for (int j = 0; j < na; ++j) {
          double l = p[i + j * (d + 2)];
          if (!(l == 0.0 || l == 2.0 || l == 3.0)) return -1;
        }
        m->sP[k] = malloc(sizeof(double) * (size_t)(3 * (d + 2)));
        memset(m->sP[k], 0, sizeof(double) * (size_t)(3 * (d + 2)));
        memcpy(m->sP[k], p + i, sizeof(double) * need);
        i += need;
      } else if (m->sdist[k] == 5) {
        int64_t need = (int64_t)mm * d + mm;
        if (np < i + need) return -1;
        m->sP[k] = malloc(sizeof(double) * need);
        memcpy(m->sP[k], p + i, sizeof(double) * need);
        i += need;
      } else {
        if (np < i + d + 1) return -1;
        m->sP[k] = malloc(sizeof(double) * (d + 1));
        memcpy(m->sP[k], p + i, sizeof(double) * (d + 1));
        i += d + 1;
      }
    }
    m->sdep = 0;
    memset(m->sdg, 0, sizeof m->sdg);
    if (np > i) {  /* the dependency block: nd, then (child, parent < child, g) */
      int nd = (int)p[i];
      if ((double)nd != p[i] || nd < 0 || np < i + 1 + 3 * (int64_t)nd) return -1;
      for (int q = 0; q < nd; ++q) {
        const double* e = p + i + 1 + 3 * q;
        int k = (int)e[0], j = (int)e[1];
        if ((double)k != e[0] || (double)j != e[1] || k < 0 || k >= m->K || j < 0 || j >= k || !isfinite(e[2])) return -1;
        int child = m->sdist[k] == 3 || m->sdist[k] == 4 || m->sdist[k] == 6 || (m->sdist[k] == 2 && m->slink[k] != 1);
        if (!child || m->sdist[j] == 1) return -1;
        m->sdg[k][j] = e[2];
        m->sdep |= 1 << k;
      }
    }
  } else if (family == ORC_REGRESSION) {
    if (dy < 1 || dy > 32 || np < 5 + (int64_t)dy) return -1;
    m->d = 2;
    m->mu_s = p[0]; m->sd_s = p[1]; m->mu_i = p[2]; m->sd_i = p[3];
    m->sigma = p[4];
    double var = p[4] * p[4];
    m->inv2v = 1.0 / (2.0 * var);
    m->cst = -0.5 * orc_log(2.0 * 0x1.921fb54442d18p+1 * var);
    m->inv2s = 1.0 / (2.0 * (p[1] * p[1]));
    m->csts = -0.5 * orc_log(2.0 * 0x1.921fb54442d18p+1 * (p[1] * p[1]));
    m->inv2i = 1.0 / (2.0 * (p[3] * p[3]));
    m->csti = -0.5 * orc_log(2.0 * 0x1.921fb54442d18p+1 * (p[3] * p[3]));
    for (int i = 0; i < dy; ++i) m->xs[i] = p[5 + i];
  } else {
    return -1;
  }
  return 0;
}

/* per-step host preprocessing of the observation */
typedef struct {
  int present;
  double bt[64];  /* LGSSM: L_R^{-1}(y - c); Kitagawa: y; HMM: symbol */
  double ct;      /* Kitagawa: 8 cos(1.2 t) */
  /* LGSSM optimal proposal: t = 1: mean mu1 (g) and constant weight w0;
     t >= 2: g = F b + K (y - c), vt = L_S^{-1}(y - c) - L_S^{-1} H b */
  double g[64], vt[64], w0;
  double raw[64]; /* the observation as given (rebuilt under other parameters: orc_pf_step_params) */
  int nraw;
  double sdk[4];  /* slot models: each dependent slot's parent term (NaN when a parent is not constrained) */
} obs_t;

static void obs_build(const model_t* m, int t, const double* y, int has, obs_t* o) {
  o->present = has;
  o->ct = 0.0;
  o->nraw = 0;
  if (m->family == ORC_KITAGAWA || (m->family == ORC_SLOTS && m->lat == 1)) o->ct = 8.0 * orc_cos(1.2 * (double)t);
  if (m->family == ORC_SLOTS && m->uin)
    for (int i = 0; i < m->d; ++i) o->bt[m->snv + i] = 0.0;  /* no input given: u_t = 0 */
  if (!has) return;
  if (m->family == ORC_SLOTS) {  /* (the engine's make_obs_slots) */
    const int inp = m->uin && ((has >> 4) & 1);  /* bit 4: the step's input follows the dy values */
    o->nraw = m->dy + (inp ? m->d : 0);
    for (int i = 0; i < o->nraw; ++i) o->raw[i] = y[i];
    if (inp)
      for (int i = 0; i < m->d; ++i) o->bt[m->snv + i] = y[m->dy + i];
    for (int k = 0; k < m->K; ++k) {
      if (!((has >> k) & 1)) continue;
      const double* yk = y + m->syoff[k];
      double* v = o->bt + m->svoff[k];
      if (m->sdist[k] == 1) {
        int mm = m->sm[k], d = m->d;
        double r[32];
        const double* c = m->sP[k] + 2 * mm * d;
        for (int j = 0; j < mm; ++j) r[j] = yk[j] - c[j];
        fwdsub(mm, 1, c + mm, r, v);
      } else if (m->sdist[k] == 3) {
        v[0] = yk[0];
        v[1] = orc_lgamma(yk[0] + 1.0);
      } else {
        v[0] = yk[0];
      }
    }
    for (int k = 0; k < m->K; ++k) {  /* the parent terms (make_obs_slots' fma chain) */
      o->sdk[k] = 0.0;
      if (!((m->sdep >> k) & 1) || !((has >> k) & 1)) continue;
      for (int j = 0; j < k; ++j) {
        if (m->sdg[k][j] == 0.0) continue;
        o->sdk[k] = ((has >> j) & 1) ? fma(m->sdg[k][j], o->bt[m->svoff[j]], o->sdk[k]) : NAN;
      }
    }
    return;
  }
  o->nraw = (m->family == ORC_LGSSM || m->family == ORC_REGRESSION) ? m->dy : 1;
  for (int i = 0; i < o->nraw; ++i) o->raw[i] = y[i];
  if (m->family == ORC_LGSSM) {
    double r[64];
    for (int i = 0; i < m->dy; ++i) r[i] = y[i] - m->c[i];
    fwdsub(m->dy, 1, m->LR, r, o->bt);
    if (m->opt) {
      int d = m->d, dy = m->dy;
      if (t == 1) {
        double e[64] = {0}, u[64] = {0}, quad = 0.0;
        for (int q = 0; q < dy; ++q) {
          double acc = r[q];
          for (int j = 0; j < d; ++j) acc = fma(-m->H[q * d + j], m->mu0[j], acc);
          e[q] = acc;
        }
        fwdsub(dy, 1, m->LS1, e, u);
        for (int q = 0; q < dy; ++q) quad = fma(u[q], u[q], quad);
        o->w0 = m->cstS1 - 0.5 * quad;
        for (int i = 0; i < d; ++i) {
          double acc = m->mu0[i];
          for (int q = 0; q < dy; ++q) acc = fma(m->Kt1[q * d + i], e[q], acc);
          o->g[i] = acc;
        }
      } else {
        double ls[64];
        fwdsub(dy, 1, m->LS, r, ls);
        for (int i = 0; i < d; ++i) {
          double acc = 0.0;
          for (int q = 0; q < dy; ++q) acc = fma(m->Kt[q * d + i], r[q], acc);
          o->g[i] = m->Fb[i] + acc;
        }
        for (int q = 0; q < dy; ++q) o->vt[q] = ls[q] - m->Wb[q];
      }
    }
  } else if (m->family == ORC_REGRESSION) {
    for (int i = 0; i < m->dy; ++i) o->bt[i] = y[i];
  } else {
    o->bt[0] = y[0];
  }
}

static double lgssm_obs(const model_t* m, const double* x, const obs_t* o) {
  if (!o->present) return 0.0;
  double quad = 0.0;
  if (m->m_diag) {
    for (int r = 0; r < m->dy; ++r) {
      double acc = fma(-m->M[r * m->d + r], x[r], o->bt[r]);
      quad = fma(acc, acc, quad);
    }
    return m->cstR - 0.5 * quad;
  }
  for (int r = 0; r < m->dy; ++r) {
    double acc = o->bt[r];
    for (int j = 0; j < m->d; ++j) acc = fma(-m->M[r * m->d + j], x[j], acc);
    quad = fma(acc, acc, quad);
  }
  return m->cstR - 0.5 * quad;
}

static int cat_sample(const double* p, int K, int stride, double u) {
  double total = 0.0;
  for (int k = 0; k < K; ++k) total += p[k * stride];
  double target = u * total;
  double cum = 0.0;
  int last = -1;
  for (int k = 0; k < K; ++k) {
    double pk = p[k * stride];
    cum += pk;
    if (pk > 0.0) last = k;
    if (cum > target && pk > 0.0) return k;
  }
  return last;
}

/* generate at t = 1: writes x[d], returns the log weight */
/* sum_i normal(y_i; slope x_i + intercept, sigma) logpdf, in data order */
static double reg_loglik(const model_t* m, const obs_t* o, const double* x) {
  if (!o->present) return 0.0;
  double s = 0.0;
  for (int i = 0; i < m->dy; ++i) {
    double diff = o->bt[i] - (x[0] * m->xs[i] + x[1]);
    s += -(diff * diff) * m->inv2v + m->cst;
  }
  return s;
}

/* draws come from (stream, base + j): the filter uses (S_INIT / S_STEP, 0),
   rejuvenation moves (S_MH, 16 * move) */
/* Gaussian custom proposal of the nonlinear SSM (particle_filter.jl:79-91,
   139-154 via trace_translators.jl:775-802): x ~ q = normal(mu_q, sigma_q),
   mu_q = alpha * m + beta * y + gamma with m the prior mean (beta * y only
   when y is observed); weight = log p(x | prior) + log p(y | x) - log q(x)
   (gen_amd/csrc/gh_models.h KitGaussModel, same operation order). */
static double kit_lpn(double x, double mu, double inv2, double cst) {
  double d = x - mu;
  return -(d * d) * inv2 + cst;
}
static double kit_gauss(const model_t* m, const obs_t* o, double mean, double inv2p, double cstp, double z,
                        double* x) {
  double mq = m->qa[0] * mean;
  if (o->present) mq = mq + m->qa[1] * o->bt[0];
  mq = mq + m->qa[2];
  x[0] = mq + m->qa[3] * z;
  double w = kit_lpn(x[0], mean, inv2p, cstp);
  if (o->present) {
    double diff = o->bt[0] - x[0] * x[0] / 20.0;
    w = w + (-(diff * diff) * m->inv2vy + m->csty);
  }
  return w - kit_lpn(x[0], mq, m->qa[4], m->qa[5]);
}

/* The nonlinear SSM's latent draw: particles p and p + 64 of every 128-particle
   group share one counter block (id ((p >> 7) << 6) | (p & 63)) and its
   Box–Muller pair, z0 for p and z1 for p + 64. */
static double kit_z(uint64_t seed, uint64_t pid, uint32_t t, uint32_t stream, uint32_t base) {
  uint32_t w[4];
  rng(seed, ((pid >> 7) << 6) | (pid & 63), t, stream, base, w);
  double z0, z1;
  box_muller(w[0], w[1], w[2], &z0, &z1);
  return ((pid >> 6) & 1) ? z1 : z0;
}

static void model_score(const model_t* m, const obs_t* o, int t, const double* xp, const double* x, double* lat,
                        double* ob);

/* The linear proposal's draw x = u (+ P xp) + L_q z and its logpdf at x (the
   mean recomputed in the same order, forward substitution with L_q) */
static double lin_draw(const model_t* m, const double* xp, const double* z, double* x) {
  const int d = m->d;
  for (int i = 0; i < d; ++i) {
    double acc = m->qu[i];
    if (xp)
      for (int k = 0; k < d; ++k) acc = fma(m->QP[i * d + k], xp[k], acc);
    for (int k = 0; k <= i; ++k) acc = fma(m->QL[i * d + k], z[k], acc);
    x[i] = acc;
  }
  double w[64], quad = 0.0;
  for (int i = 0; i < d; ++i) {
    double mean = m->qu[i];
    if (xp)
      for (int k = 0; k < d; ++k) mean = fma(m->QP[i * d + k], xp[k], mean);
    double r = x[i] - mean;
    for (int k = 0; k < i; ++k) r = fma(-m->QL[i * d + k], w[k], r);
    w[i] = r / m->QL[i * d + i];
    quad = fma(w[i], w[i], quad);
  }
  return m->cstq - 0.5 * quad;
}

/* ---- the slot family (gen_amd/csrc/gh_slots.h SlotModel, line for line) */
/* a draw's counter: (seed, id, 0, S_DIST, draw) for the distribution entry
   points, (seed, particle, t, S_SIM, base + draw) for a slot model's simulate */
typedef struct { uint64_t seed, id; uint32_t t, stream, base; } od_rng;
static double od_logpdf(int dist, const double* x, int64_t xs, const double* P, int D, int K);
static void od_random(int dist, const od_rng* r, double* x, int64_t xs, const double* P, int D, int K);
#define SLOT_LIB_DRAW 1024u /* simulate(): library slot k draws from SLOT_LIB_DRAW + 256 k */
static double slot_affine(const double* h, double c, const double* x, int d) {
  double acc = c;
  for (int j = 0; j < d; ++j) acc = fma(h[j], x[j], acc);
  return acc;
}
/* normal.jl:56-60 with std = exp(eta): var = std * std, -(diff^2) / (2 var) - 0.5 log(2 pi var) */
static double slot_logscale_lpdf(double diff, double eta) {
  double sd = orc_exp(eta);
  double var = sd * sd;
  return -(diff * diff) / (2.0 * var) - 0.5 * orc_log(0x1.921fb54442d18p+2 * var);
}
static double slot_link(int link, double eta) {
  return link == 2 ? orc_exp(eta) : (link == 3 ? 1.0 / (1.0 + orc_exp(-eta)) : eta);
}
static double slot_eta(const model_t* m, const double* h, double c, const double* x, int k, double dk);
static void slot_lib_args(const model_t* m, const double* P, int na, const double* x, int k, double dk, double a[3]) {
  const int d = m->d;
  for (int j = 0; j < 3; ++j) {
    const double* B = P + j * (d + 2);
    a[j] = j < na ? slot_link((int)B[0], j == 0 ? slot_eta(m, B + 1, B[d + 1], x, k, dk) : slot_affine(B + 1, B[d + 1], x, d))
                  : 0.0;
  }
}
/* c + h.x, plus slot k's parent term when it has parents (SlotModel::eta) */
static double slot_eta(const model_t* m, const double* h, double c, const double* x, int k, double dk) {
  double e = slot_affine(h, c, x, m->d);
  return ((m->sdep >> k) & 1) ? e + dk : e;
}
static double slot_lpdf_d(const model_t* m, const double* v, int k, const double* x, double dk);
static double slot_lpdf(const model_t* m, const obs_t* o, int k, const double* x) {
  return slot_lpdf_d(m, o->bt + m->svoff[k], k, x, ((m->sdep >> k) & 1) ? o->sdk[k] : 0.0);
}
static double slot_lpdf_d(const model_t* m, const double* v, int k, const double* x, double dk) {
  const int d = m->d, mm = m->sm[k];
  const double* P = m->sP[k];
  switch (m->sdist[k]) {
    case 6: {  /* the library's logpdf (od_logpdf: the reference's formulas) */
      double a[3];
      slot_lib_args(m, P, slot_lib_nargs(mm), x, k, dk, a);
      return od_logpdf(mm, v, 1, a, 1, 0);
    }
    case 1: {  /* mvnormal(H x + c, R) through L_R^-1 (y - c) (mvnormal.jl:12-16) */
      double quad = 0.0;
      for (int r = 0; r < mm; ++r) {
        double acc = v[r];
        for (int j = 0; j < d; ++j) acc = fma(-P[r * d + j], x[j], acc);
        quad = fma(acc, acc, quad);
      }
      return m->scst[k] - 0.5 * quad;
    }
    case 2: {  /* normal.jl:56-60 */
      double mean = m->slink[k] == 1 ? x[0] * x[0] / 20.0 : slot_eta(m, P, P[d], x, k, dk);
      double diff = v[0] - mean;
      if (m->slink[k] == 5) return slot_logscale_lpdf(diff, slot_affine(P + d + 1, P[2 * d + 1], x, d));
      return -(diff * diff) * m->sinv2v[k] + m->scst[k];
    }
    case 3: {  /* poisson.jl:10-12, lambda = exp(h.x + c) */
      double lam = orc_exp(slot_eta(m, P, P[d], x, k, dk));
      return v[0] < 0.0 ? -INFINITY : (v[0] * orc_log(lam) - lam) - v[1];
    }
    case 4: {  /* bernoulli.jl:10-12, prob = 1 / (1 + exp(-(h.x + c))) */
      double prob = 1.0 / (1.0 + orc_exp(-slot_eta(m, P, P[d], x, k, dk)));
      return v[0] != 0.0 ? orc_log(prob) : orc_log(1.0 - prob);
    }
    default: {  /* categorical.jl:10-12, probs = exp(eta - max eta) / sum (0-based value) */
      double mx = -INFINITY, s = 0.0, ey = 0.0;
      for (int j = 0; j < mm; ++j) mx = fmax(mx, slot_affine(P + j * d, P[mm * d + j], x, d));
      int y = (int)v[0];
      for (int j = 0; j < mm; ++j) {
        double e = orc_exp(slot_affine(P + j * d, P[mm * d + j], x, d) - mx);
        s += e;
        if (j == y) ey = e;
      }
      return orc_log(ey / s);
    }
  }
}
static double slot_loglik(const model_t* m, const obs_t* o, const double* x) {
  double w = 0.0;
  for (int k = 0; k < m->K; ++k)
    if ((o->present >> k) & 1) w = w + slot_lpdf(m, o, k, x);
  return w;
}
static double kit_z(uint64_t seed, uint64_t pid, uint32_t t, uint32_t stream, uint32_t base);
/* the latent of step t (t = 1: the initial distribution), dense forms */
/* the class of a one-hot categorical latent (SlotModel::onehot) */
static int slot_onehot(const double* x, int d) {
  int z = 0;
  for (int j = 0; j < d; ++j) z = x[j] != 0.0 ? j : z;
  return z;
}
/* the regime of a switching state (its one-hot tail, SlotModel::regime) */
static int slot_regime(const model_t* m, const double* x) {
  int dx = m->d - m->nz, z = 0;
  for (int j = dx; j < m->d; ++j) z = x[j] != 0.0 ? j - dx : z;
  return z;
}
static void slot_latent(const model_t* m, uint64_t seed, uint64_t pid, uint32_t t, const obs_t* o,
                        const double* xp, double* x, uint32_t stream, uint32_t base) {
  if (m->lat == 4) {  /* the regime (inverse CDF, draw base), then x under it (normals from base + 1) */
    uint32_t w[4];
    rng(seed, pid, t, stream, base, w);
    const double u = unif53(w[0], w[1]);
    const int nz = m->nz, d = m->d, dx = d - nz;
    const int z = t == 1 ? cat_sample(m->prior, nz, 1, u) : cat_sample(m->T + slot_regime(m, xp), nz, nz, u);
    const double* blk = m->SW + z * (2 * dx * dx + dx);
    const double* L = t == 1 ? m->L0 : blk + dx * dx + dx;
    double zn[64];
    normals_at(seed, pid, t, stream, base + 1, d, zn);
    for (int i = 0; i < d; ++i) {
      if (i < dx) {
        double acc;
        if (t == 1) {
          acc = m->mu0[i];
        } else {
          acc = blk[dx * dx + i];
          for (int k = 0; k < dx; ++k) acc = fma(blk[i * dx + k], xp[k], acc);
        }
        for (int k = 0; k <= i; ++k) acc = fma(L[i * dx + k], zn[k], acc);
        x[i] = acc;
      } else {
        x[i] = i - dx == z ? 1.0 : 0.0;
      }
    }
    return;
  }
  if (m->lat == 3) {  /* inverse-CDF draw (categorical.jl:20-22), as the HMM family's */
    uint32_t w[4];
    rng(seed, pid, t, stream, base, w);
    const double u = unif53(w[0], w[1]);
    const int d = m->d;
    const int z = t == 1 ? cat_sample(m->prior, d, 1, u) : cat_sample(m->T + slot_onehot(xp, d), d, d, u);
    for (int j = 0; j < d; ++j) x[j] = j == z ? 1.0 : 0.0;
    return;
  }
  if (m->lat == 1) {
    double z = kit_z(seed, pid, t, stream, base);
    if (t == 1) x[0] = m->mu1 + m->s1 * z;
    else {
      double v = xp[0];
      x[0] = (((v / 2.0) + 25.0 * (v / (1.0 + v * v))) + o->ct) + m->sx * z;
    }
    return;
  }
  int d = m->d;
  double z[64];
  normals_at(seed, pid, t, stream, base, d, z);
  for (int i = 0; i < d; ++i) {
    double acc;
    if (t == 1) {
      acc = m->mu0[i];
      for (int k = 0; k <= i; ++k) acc = fma(m->L0[i * d + k], z[k], acc);
    } else {
      acc = m->uin ? m->b[i] + o->bt[m->snv + i] : m->b[i];
      for (int k = 0; k < d; ++k) acc = fma(m->A[i * d + k], xp[k], acc);
      for (int k = 0; k <= i; ++k) acc = fma(m->LQ[i * d + k], z[k], acc);
    }
    x[i] = acc;
  }
}
/* poisson_chop of gh_dists.h: chop-down inversion from the mode with one uniform */
static double slot_poisson_chop(double lam, double u) {
  if (lam == 0.0) return 0.0;
  if (!(lam > 0.0) || lam == INFINITY) return NAN;
  double m = floor(lam);
  double pm = orc_exp((m == 0.0 ? 0.0 : m * orc_log(lam)) - lam - orc_lgamma(m + 1.0));
  u -= pm;
  if (u <= 0.0) return m;
  double lo = m, hi = m, pl = pm, ph = pm;
  for (int it = 0; it < (1 << 24); ++it) {
    hi += 1.0; ph = ph * lam / hi; u -= ph;
    if (u <= 0.0) return hi;
    if (lo > 0.0) { pl = pl * lo / lam; lo -= 1.0; u -= pl; if (u <= 0.0) return lo; }
    if (ph == 0.0 && (lo <= 0.0 || pl == 0.0)) break;
  }
  return m;
}
/* simulate(): every slot's value (slot k from draws SIM_OBS_DRAW + 32 k), in
   the observation vector's layout */
static void slot_sim(const model_t* m, uint64_t seed, uint64_t pid, uint32_t t, const double* x, double* y) {
  const int d = m->d;
  double ysc[4];  /* the scalar slots' draws (parents of later slots) */
  for (int k = 0; k < m->K; ++k) {
    const int mm = m->sm[k];
    double dk = 0.0;  /* the parent term (SlotModel::sim_obs) */
    if ((m->sdep >> k) & 1)
      for (int j = 0; j < k; ++j)
        if (m->sdg[k][j] != 0.0) dk = fma(m->sdg[k][j], ysc[j], dk);
    const uint32_t draw = 32u + 32u * (uint32_t)k;
    const double* P = m->sP[k];
    double* yk = y + m->syoff[k];
    uint32_t w[4];
    if (m->sdist[k] == 6) {
      double a[3];
      slot_lib_args(m, P, slot_lib_nargs(mm), x, k, dk, a);
      const od_rng r = {seed, pid, t, 7, SLOT_LIB_DRAW + 256u * (uint32_t)k};
      od_random(mm, &r, yk, 1, a, 1, 0);
    } else if (m->sdist[k] == 1) {
      const double *H = P + mm * d, *c = H + mm * d, *LR = c + mm;
      double z[32];
      normals_at(seed, pid, t, 7, draw, mm, z);
      for (int r = 0; r < mm; ++r) {
        double acc = c[r];
        for (int j = 0; j < d; ++j) acc = fma(H[r * d + j], x[j], acc);
        for (int q = 0; q <= r; ++q) acc = fma(LR[r * mm + q], z[q], acc);
        yk[r] = acc;
      }
    } else if (m->sdist[k] == 2) {
      double z[2];
      normals_at(seed, pid, t, 7, draw, 1, z);
      double mean = m->slink[k] == 1 ? x[0] * x[0] / 20.0 : slot_eta(m, P, P[d], x, k, dk);
      double sd = m->slink[k] == 5 ? orc_exp(slot_affine(P + d + 1, P[2 * d + 1], x, d)) : m->ssd[k];
      yk[0] = mean + sd * z[0];
    } else if (m->sdist[k] == 3) {
      rng(seed, pid, t, 7, draw, w);
      yk[0] = slot_poisson_chop(orc_exp(slot_eta(m, P, P[d], x, k, dk)), unif53(w[0], w[1]));
    } else if (m->sdist[k] == 4) {
      rng(seed, pid, t, 7, draw, w);
      double prob = 1.0 / (1.0 + orc_exp(-slot_eta(m, P, P[d], x, k, dk)));
      yk[0] = unif53(w[0], w[1]) < prob ? 1.0 : 0.0;
    } else {
      rng(seed, pid, t, 7, draw, w);
      double e[16], mx = -INFINITY;
      for (int j = 0; j < mm; ++j) mx = fmax(mx, slot_affine(P + j * d, P[mm * d + j], x, d));
      for (int j = 0; j < mm; ++j) e[j] = orc_exp(slot_affine(P + j * d, P[mm * d + j], x, d) - mx);
      yk[0] = (double)cat_sample(e, mm, 1, unif53(w[0], w[1]));
    }
    ysc[k] = yk[0];
  }
}

static double particle_init(const model_t* m, uint64_t seed, uint64_t pid, const obs_t* o,
                            int proposal, double* x, uint32_t stream, uint32_t base) {
  if (m->family == ORC_SLOTS) {
    if (proposal == ORC_PROPOSAL_LINEAR) {  /* custom proposal: model weight - proposal score */
      double z[64];
      normals_at(seed, pid, 1, stream, base, m->d, z);
      const double lq = lin_draw(m, NULL, z, x);
      double lat, ob;
      model_score(m, o, 1, x, x, &lat, &ob);
      return (lat + ob) - lq;
    }
    slot_latent(m, seed, pid, 1, o, NULL, x, stream, base);
    return slot_loglik(m, o, x);
  }
  if (m->family == ORC_REGRESSION) {
    double z[2];
    normals_at(seed, pid, 1, stream, base, 2, z);
    x[0] = m->mu_s + m->sd_s * z[0];
    x[1] = m->mu_i + m->sd_i * z[1];
    return reg_loglik(m, o, x);
  }
  if (m->family == ORC_LGSSM) {
    double z[64];
    normals_at(seed, pid, 1, stream, base, m->d, z);
    if (proposal == ORC_PROPOSAL_LINEAR) {  /* custom proposal: model weight - proposal score */
      const double lq = lin_draw(m, NULL, z, x);
      double lat, ob;
      model_score(m, o, 1, x, x, &lat, &ob);
      return (lat + ob) - lq;
    }
    if (proposal == ORC_PROPOSAL_OPTIMAL && o->present) {
      /* x ~ N(mu1, (I - K1 H) P0); weight log N(y; H mu0 + c, H P0 H^T + R) */
      for (int i = 0; i < m->d; ++i) {
        double acc = o->g[i];
        for (int k = 0; k <= i; ++k) acc = fma(m->LSig1[i * m->d + k], z[k], acc);
        x[i] = acc;
      }
      return o->w0;
    }
    for (int i = 0; i < m->d; ++i) {
      double acc = m->mu0[i];
      for (int k = 0; k <= i; ++k) acc = fma(m->L0[i * m->d + k], z[k], acc);
      x[i] = acc;
    }
    return lgssm_obs(m, x, o);
  } else if (m->family == ORC_KITAGAWA) {
    if (proposal == ORC_PROPOSAL_GAUSSIAN) return kit_gauss(m, o, m->mu1, m->inv2v1, m->cst1, kit_z(seed, pid, 1, stream, base), x);
    x[0] = m->mu1 + m->s1 * kit_z(seed, pid, 1, stream, base);
    if (!o->present) return 0.0;
    double diff = o->bt[0] - x[0] * x[0] / 20.0;
    return -(diff * diff) * m->inv2vy + m->csty;
  } else {
    uint32_t w[4];
    rng(seed, pid, 1, stream, base, w);
    double u = unif53(w[0], w[1]);
    int K = m->k;
    if (proposal == ORC_PROPOSAL_OPTIMAL && o->present) {
      int xs = (int)o->bt[0];
      double p[64];
      for (int kk = 0; kk < K; ++kk) p[kk] = m->prior[kk] * m->E[xs * K + kk];
      double total = 0.0;
      for (int kk = 0; kk < K; ++kk) total += p[kk];
      x[0] = (double)cat_sample(p, K, 1, u);
      return orc_log(total);
    }
    int z = cat_sample(m->prior, K, 1, u);
    x[0] = (double)z;
    return o->present ? m->logE[(int)o->bt[0] * K + z] : 0.0;
  }
}

/* update at step t >= 2 from previous latent xp: writes x, returns increment */
static double particle_step(const model_t* m, uint64_t seed, uint64_t pid, uint32_t t,
                            const obs_t* o, int proposal, const double* xp, double* x, uint32_t stream,
                            uint32_t base) {
  if (m->family == ORC_SLOTS) {
    if (proposal == ORC_PROPOSAL_LINEAR) {
      double z[64];
      normals_at(seed, pid, t, stream, base, m->d, z);
      const double lq = lin_draw(m, xp, z, x);
      double lat, ob;
      model_score(m, o, (int)t, xp, x, &lat, &ob);
      return (lat + ob) - lq;
    }
    slot_latent(m, seed, pid, t, o, xp, x, stream, base);
    return slot_loglik(m, o, x);
  }
  if (m->family == ORC_LGSSM) {
    double z[64];
    normals_at(seed, pid, t, stream, base, m->d, z);
    int d = m->d;
    if (proposal == ORC_PROPOSAL_LINEAR) {
      const double lq = lin_draw(m, xp, z, x);
      double lat, ob;
      model_score(m, o, (int)t, xp, x, &lat, &ob);
      return (lat + ob) - lq;
    }
    if (proposal == ORC_PROPOSAL_OPTIMAL && o->present) {
      /* x ~ N(F A xp + g, Sigma); weight log p(y | xp) = log N(y; H (A xp + b) + c, S) */
      for (int i = 0; i < d; ++i) {
        double acc = o->g[i];
        for (int k = 0; k < d; ++k) acc = fma(m->FA[i * d + k], xp[k], acc);
        for (int k = 0; k <= i; ++k) acc = fma(m->LSig[i * d + k], z[k], acc);
        x[i] = acc;
      }
      double quad = 0.0;
      for (int r = 0; r < m->dy; ++r) {
        double u = o->vt[r];
        for (int k = 0; k < d; ++k) u = fma(-m->WA[r * d + k], xp[k], u);
        quad = fma(u, u, quad);
      }
      return m->cstS - 0.5 * quad;
    }
    for (int i = 0; i < d; ++i) {
      double acc = m->b[i];
      for (int k = 0; k < d; ++k) acc = fma(m->A[i * d + k], xp[k], acc);
      /* the optimal proposal without an observation is the prior in its dense
         form (the engine's LGOptModel<D> falls back to LGModel<D, 0>) */
      if (m->lq_diag && proposal != ORC_PROPOSAL_OPTIMAL) acc = fma(m->LQ[i * d + i], z[i], acc);
      else for (int k = 0; k <= i; ++k) acc = fma(m->LQ[i * d + k], z[k], acc);
      x[i] = acc;
    }
    return lgssm_obs(m, x, o);
  } else if (m->family == ORC_KITAGAWA) {
    double v = xp[0];
    double mean = ((v / 2.0) + 25.0 * (v / (1.0 + v * v))) + o->ct;
    if (proposal == ORC_PROPOSAL_GAUSSIAN) return kit_gauss(m, o, mean, m->inv2vx, m->cstx, kit_z(seed, pid, t, stream, base), x);
    x[0] = mean + m->sx * kit_z(seed, pid, t, stream, base);
    if (!o->present) return 0.0;
    double diff = o->bt[0] - x[0] * x[0] / 20.0;
    return -(diff * diff) * m->inv2vy + m->csty;
  } else {
    uint32_t w[4];
    rng(seed, pid, t, stream, base, w);
    double u = unif53(w[0], w[1]);
    int K = m->k, zp = (int)xp[0];
    if (proposal == ORC_PROPOSAL_OPTIMAL && o->present) {
      int xs = (int)o->bt[0];
      double p[64];
      for (int kk = 0; kk < K; ++kk) p[kk] = m->T[kk * K + zp] * m->E[xs * K + kk];
      double total = 0.0;
      for (int kk = 0; kk < K; ++kk) total += p[kk];
      x[0] = (double)cat_sample(p, K, 1, u);
      return orc_log(total);
    }
    int z = cat_sample(m->T + zp, K, K, u);
    x[0] = (double)z;
    return o->present ? m->logE[(int)o->bt[0] * K + z] : 0.0;
  }
}

/* ---------------------------------------------------------- PF state */
struct orc_pf {
  model_t m;
  int64_t n_global, lo, n;
  uint64_t seed;
  int resampler, record_history;
  int t;                /* number of completed steps (1 after init) */
  double* x;            /* [d][n] current */
  double* xprev;        /* [d][n] scratch */
  double* logw;
  int64_t* anc;         /* pending ancestors (global ids) */
  double* anc_state;    /* [d][n] ancestor states after a (distributed) resample */
  int pending;          /* resampled since the last step */
  double log_ml_est;
  obs_t obs;            /* observation of the current step (rejuvenation) */
  int cond;             /* conditional SMC: particle 0 is pinned (smc.jl:100-151) */
  uint32_t moves;       /* rejuvenation moves applied at the current step */
  /* history */
  int cap;
  double** hx;
  int32_t** hanc;
  int* hres;
  obs_t* hobs;          /* every step's observation (trace scores) */
};

orc_pf* orc_pf_create(int family, int d, int dy, int k, int v, const double* params, int64_t np,
                      int64_t n_global, int64_t lo, int64_t n_local, uint64_t seed, int resampler,
                      int record_history) {
  orc_pf* pf = calloc(1, sizeof(orc_pf));
  if (model_build(&pf->m, family, d, dy, k, v, params, np)) { model_free(&pf->m); free(pf); return NULL; }
  pf->n_global = n_global; pf->lo = lo; pf->n = n_local; pf->seed = seed;
  pf->resampler = resampler; pf->record_history = record_history;
  int D = pf->m.d;
  pf->x = calloc((size_t)D * n_local, sizeof(double));
  pf->xprev = calloc((size_t)D * n_local, sizeof(double));
  pf->anc_state = calloc((size_t)D * n_local, sizeof(double));
  pf->logw = calloc((size_t)n_local, sizeof(double));
  pf->anc = calloc((size_t)n_local, sizeof(int64_t));
  return pf;
}

void orc_pf_destroy(orc_pf* pf) {
  if (!pf) return;
  for (int i = 0; i < pf->cap; ++i) { free(pf->hx[i]); free(pf->hanc[i]); }
  free(pf->hx); free(pf->hanc); free(pf->hres); free(pf->hobs);
  free(pf->x); free(pf->xprev); free(pf->anc_state); free(pf->logw); free(pf->anc);
  model_free(&pf->m);
  free(pf);
}

static void record(orc_pf* pf) {
  if (!pf->record_history) return;
  int t = pf->t;  /* 1-based step just completed */
  if (t > pf->cap) {
    int nc = pf->cap ? pf->cap * 2 : 16;
    while (nc < t) nc *= 2;
    pf->hx = realloc(pf->hx, sizeof(double*) * nc);
    pf->hanc = realloc(pf->hanc, sizeof(int32_t*) * nc);
    pf->hres = realloc(pf->hres, sizeof(int) * nc);
    pf->hobs = realloc(pf->hobs, sizeof(obs_t) * nc);
    for (int i = pf->cap; i < nc; ++i) { pf->hx[i] = NULL; pf->hanc[i] = NULL; pf->hres[i] = 0; }
    pf->cap = nc;
  }
  size_t sz = (size_t)pf->m.d * pf->n;
  pf->hx[t - 1] = malloc(sizeof(double) * sz);
  memcpy(pf->hx[t - 1], pf->x, sizeof(double) * sz);
  pf->hobs[t - 1] = pf->obs;
}

static double model_loglik(const model_t* m, const obs_t* o, const double* x);

static int init_impl(orc_pf* pf, const double* obs, int has_obs, int proposal, const double* ref) {
  obs_t o;
  obs_build(&pf->m, 1, obs, has_obs, &o);
  int D = pf->m.d;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < pf->n; ++i) {
    double x[64];
    pf->logw[i] = particle_init(&pf->m, pf->seed, (uint64_t)(pf->lo + i), &o, proposal, x, S_INIT, 0);
    for (int k = 0; k < D; ++k) pf->x[(size_t)k * pf->n + i] = x[k];
    pf->anc[i] = pf->lo + i;
  }
  if (ref) {  /* distinguished particle: given state, weight init_score (smc.jl:114-115) */
    for (int k = 0; k < D; ++k) pf->x[(size_t)k * pf->n] = ref[k];
    pf->logw[0] = model_loglik(&pf->m, &o, ref);
    pf->cond = 1;
  }
  pf->t = 1;
  pf->pending = 0;
  pf->log_ml_est = 0.0;
  pf->obs = o;
  pf->moves = 0;
  record(pf);
  return 0;
}
static int proposal_ok(const model_t* m, int proposal) {
  if (proposal == 0) return 1;
  if (proposal == ORC_PROPOSAL_GAUSSIAN) return m->family == ORC_KITAGAWA && m->qa[3] > 0.0;
  if (proposal == ORC_PROPOSAL_LINEAR)
    return m->qlin && ((m->family == ORC_LGSSM && m->d + m->dy <= 32) ||
                       (m->family == ORC_SLOTS && m->lat != 3 && m->lat != 4 && m->d + m->snv + (m->uin ? m->d : 0) <= 32));
  return proposal == ORC_PROPOSAL_OPTIMAL && (m->family == ORC_HMM || (m->family == ORC_LGSSM && m->opt));
}
int orc_pf_set_proposal_args(orc_pf* pf, const double* args, int n) {
  model_t* m = &pf->m;
  if (m->family == ORC_LGSSM || m->family == ORC_SLOTS) {  /* the linear proposal: P Sigma_q u, or u alone */
    const int d = m->d;
    if (n == d && m->qlin) {
      for (int i = 0; i < d; ++i) m->qu[i] = args[i];
      return 0;
    }
    if (n != 2 * d * d + d) return -1;
    double* L = malloc(sizeof(double) * d * d);
    if (chol(d, args + d * d, L)) { free(L); return -1; }
    free(m->QP); free(m->QL);
    m->QP = malloc(sizeof(double) * d * d);
    for (int i = 0; i < d * d; ++i) m->QP[i] = args[i];
    m->QL = L;
    m->cstq = gauss_cst(d, L);
    for (int i = 0; i < d; ++i) m->qu[i] = args[2 * d * d + i];
    m->qlin = 1;
    return 0;
  }
  if (n != 4 || !(args[3] > 0.0)) return -1;
  double v = args[3] * args[3];
  pf->m.qa[0] = args[0]; pf->m.qa[1] = args[1]; pf->m.qa[2] = args[2]; pf->m.qa[3] = args[3];
  pf->m.qa[4] = 1.0 / (2.0 * v);
  pf->m.qa[5] = -0.5 * orc_log(2.0 * 0x1.921fb54442d18p+1 * v);
  return 0;
}
int orc_pf_init(orc_pf* pf, const double* obs, int has_obs, int proposal) {
  if (!proposal_ok(&pf->m, proposal)) return -1;
  return init_impl(pf, obs, has_obs, proposal, NULL);
}
int orc_pf_init_conditional(orc_pf* pf, const double* obs, int has_obs, const double* ref) {
  if (pf->resampler != ORC_MULTINOMIAL || pf->lo != 0 || pf->n != pf->n_global) return -1;
  return init_impl(pf, obs, has_obs, 0, ref);
}

static int step_impl(orc_pf* pf, const double* obs, int has_obs, int proposal, const double* ref) {
  if (pf->m.family == ORC_REGRESSION) return -1; /* a static model has no steps */
  uint32_t t = (uint32_t)(pf->t + 1);
  obs_t o;
  obs_build(&pf->m, (int)t, obs, has_obs, &o);
  int D = pf->m.d;
  int64_t n = pf->n;
  double* src = pf->pending ? pf->anc_state : pf->x;
  memcpy(pf->xprev, src, sizeof(double) * D * n);
  const double w0_old = n > 0 ? pf->logw[0] : 0.0;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    double xp[64], x[64];
    for (int k = 0; k < D; ++k) xp[k] = pf->xprev[(size_t)k * n + i];
    double inc = particle_step(&pf->m, pf->seed, (uint64_t)(pf->lo + i), t, &o, proposal, xp, x, S_STEP, 0);
    for (int k = 0; k < D; ++k) pf->x[(size_t)k * n + i] = x[k];
    pf->logw[i] = (pf->pending ? 0.0 : pf->logw[i]) + inc;
  }
  if (ref) {  /* distinguished particle: parent itself, weight += forward_score (smc.jl:138-141) */
    for (int k = 0; k < D; ++k) pf->x[(size_t)k * n] = ref[k];
    pf->logw[0] = (pf->pending ? 0.0 : w0_old) + model_loglik(&pf->m, &o, ref);
  }
  int was = pf->pending;
  pf->pending = 0;
  pf->t = (int)t;
  pf->obs = o;
  pf->moves = 0;
  record(pf);
  if (pf->record_history) {
    pf->hres[t - 1] = was;
    if (was) {
      pf->hanc[t - 1] = malloc(sizeof(int32_t) * n);
      for (int64_t i = 0; i < n; ++i) pf->hanc[t - 1][i] = (int32_t)pf->anc[i];
    }
  }
  return 0;
}

int orc_pf_step(orc_pf* pf, const double* obs, int has_obs, int proposal) {
  if (pf->cond || !proposal_ok(&pf->m, proposal)) return -1;
  return step_impl(pf, obs, has_obs, proposal, NULL);
}
int orc_pf_step_conditional(orc_pf* pf, const double* obs, int has_obs, const double* ref) {
  if (!pf->cond) return -1;
  return step_impl(pf, obs, has_obs, 0, ref);
}

/* log p(y_t | x_t): the step's weight increment under the prior proposal */
static double model_loglik(const model_t* m, const obs_t* o, const double* x) {
  if (m->family == ORC_SLOTS) return slot_loglik(m, o, x);
  if (m->family == ORC_LGSSM) return lgssm_obs(m, x, o);
  if (m->family == ORC_REGRESSION) return reg_loglik(m, o, x);
  if (!o->present) return 0.0;
  if (m->family == ORC_KITAGAWA) {
    double diff = o->bt[0] - x[0] * x[0] / 20.0;
    return -(diff * diff) * m->inv2vy + m->csty;
  }
  return m->logE[(int)o->bt[0] * m->k + (int)x[0]];
}

/* Rejuvenation: mh(trace, select(x_t)) on every particle (src/inference/mh.jl:14-26):
   regenerate x_t from its prior given the parent state x_{t-1} (the states the
   last step read, pf->xprev), weight = log p(y|x') - log p(y|x), accept iff
   log(u) < weight.  Move w of the step uses stream S_MH + 16 (w / 4096), draws
   [16 (w mod 4096), +8) for the proposal and draw 16 (w mod 4096) + 15 for u. */
int orc_pf_rejuvenate(orc_pf* pf, int n_moves, int64_t* accepted) {
  return orc_pf_mh_select(pf, pf->m.family == ORC_REGRESSION ? 3u : 1u, n_moves, accepted);
}

/* mh(trace, selection) on every particle (src/inference/mh.jl:14-28): the
   regression regenerates the selected ones of :slope (bit 0) / :intercept
   (bit 1) with the same draws as a full regeneration, weight = the
   log-likelihood difference (quickstart.jl:17-22); the Unfold families have
   one latent address per step (the rejuvenation move above). */
int orc_pf_mh_select(orc_pf* pf, uint32_t mask, int n_moves, int64_t* accepted) {
  const uint32_t all = pf->m.family == ORC_REGRESSION ? 3u : 1u;
  if (mask == 0 || (mask & ~all)) return -1;
  if (pf->m.family == ORC_REGRESSION && pf->t != 1) return -1;
  if (pf->cond || pf->pending || pf->t < 1 || n_moves < 0 || (uint64_t)pf->moves + (uint64_t)n_moves > (1u << 24)) return -1;
  const int D = pf->m.d;
  const int64_t n = pf->n;
  const uint32_t t = (uint32_t)pf->t;
  int64_t acc = 0;
  double x[64], xp[64], y[64];
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t pid = (uint64_t)(pf->lo + i);
    for (int k = 0; k < D; ++k) x[k] = pf->x[(size_t)k * n + i];
    if (t >= 2)
      for (int k = 0; k < D; ++k) xp[k] = pf->xprev[(size_t)k * n + i];
    double ll = model_loglik(&pf->m, &pf->obs, x);
    for (int m = 0; m < n_moves; ++m) {
      const uint32_t mv = pf->moves + (uint32_t)m;
      const uint32_t stream = (uint32_t)S_MH + ((mv >> 12) << 4), base = (mv & 4095u) * 16u;
      double ll2 = t == 1 ? particle_init(&pf->m, pf->seed, pid, &pf->obs, 0, y, stream, base)
                          : particle_step(&pf->m, pf->seed, pid, t, &pf->obs, 0, xp, y, stream, base);
      if (pf->m.family == ORC_REGRESSION && mask != all) {
        if (!(mask & 1u)) y[0] = x[0];
        if (!(mask & 2u)) y[1] = x[1];
        ll2 = reg_loglik(&pf->m, &pf->obs, y);
      }
      uint32_t w[4];
      rng(pf->seed, pid, t, stream, base + 15u, w);
      const double logu = orc_log(unif53(w[0], w[1]));
      if (logu < ll2 - ll) {
        for (int k = 0; k < D; ++k) x[k] = y[k];
        ll = ll2;
        ++acc;
      }
    }
    for (int k = 0; k < D; ++k) pf->x[(size_t)k * n + i] = x[k];
  }
  pf->moves += (uint32_t)n_moves;
  if (pf->record_history && pf->hx && pf->hx[t - 1])
    memcpy(pf->hx[t - 1], pf->x, sizeof(double) * (size_t)D * n);
  if (accepted) *accepted = acc;
  return 0;
}

static void model_score(const model_t* m, const obs_t* o, int t, const double* xp, const double* x, double* lat,
                        double* ob);

/* mh(trace, drift, (sd,)) on every particle (src/inference/mh.jl:41-62): the
   Gaussian drift proposal on the selected latent addresses (the Unfold
   families' x_t as a whole, the regression's :slope / :intercept by bit), the
   update weight as the acceptance ratio (the symmetric drift's forward and
   backward scores are equal); the trace scores of model_score. */
int orc_pf_mh_drift(orc_pf* pf, uint32_t mask, const double* sd_in, int n_moves, int64_t* accepted) {
  const uint32_t all = pf->m.family == ORC_REGRESSION ? 3u : 1u;
  if (pf->m.family == ORC_HMM || mask == 0 || (mask & ~all)) return -1;
  if (pf->m.family == ORC_REGRESSION && pf->t != 1) return -1;
  if (pf->cond || pf->pending || pf->t < 1 || n_moves < 0 || (uint64_t)pf->moves + (uint64_t)n_moves > (1u << 24)) return -1;
  const int D = pf->m.d;
  double sd[64];
  for (int k = 0; k < D; ++k) {
    int sel = pf->m.family == ORC_REGRESSION ? (int)((mask >> k) & 1u) : 1;
    if (sel && !(sd_in[k] > 0.0 && sd_in[k] < INFINITY)) return -1;
    sd[k] = sel ? sd_in[k] : 0.0;
  }
  const int64_t n = pf->n;
  const uint32_t t = (uint32_t)pf->t;
  int64_t acc = 0;
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t pid = (uint64_t)(pf->lo + i);
    double x[64], xp[64] = {0}, y[64], z[64], lat, ob;
    for (int k = 0; k < D; ++k) x[k] = pf->x[(size_t)k * n + i];
    if (t >= 2)
      for (int k = 0; k < D; ++k) xp[k] = pf->xprev[(size_t)k * n + i];
    model_score(&pf->m, &pf->obs, (int)t, xp, x, &lat, &ob);
    double s = lat + ob;
    for (int m = 0; m < n_moves; ++m) {
      const uint32_t mv = pf->moves + (uint32_t)m;
      const uint32_t stream = (uint32_t)S_MH + ((mv >> 12) << 4), base = (mv & 4095u) * 16u;
      normals_at(pf->seed, pid, t, stream, base, D, z);
      for (int k = 0; k < D; ++k) y[k] = sd[k] > 0.0 ? x[k] + sd[k] * z[k] : x[k];
      model_score(&pf->m, &pf->obs, (int)t, xp, y, &lat, &ob);
      const double s2 = lat + ob;
      uint32_t w[4];
      rng(pf->seed, pid, t, stream, base + 15u, w);
      if (orc_log(unif53(w[0], w[1])) < s2 - s) {
        for (int k = 0; k < D; ++k) x[k] = y[k];
        s = s2;
        ++acc;
      }
    }
    for (int k = 0; k < D; ++k) pf->x[(size_t)k * n + i] = x[k];
  }
  pf->moves += (uint32_t)n_moves;
  if (pf->record_history && pf->hx && pf->hx[t - 1])
    memcpy(pf->hx[t - 1], pf->x, sizeof(double) * (size_t)D * n);
  if (accepted) *accepted = acc;
  return 0;
}

void orc_pf_local_stats(orc_pf* pf, double out[3]) {
  double M = -INFINITY;
  for (int64_t i = 0; i < pf->n; ++i) {
    double w = pf->pending ? 0.0 : pf->logw[i];
    if (w > M) M = w;
  }
  double S = 0.0, S2 = 0.0;
  if (M > -INFINITY) {
    double* e = malloc(sizeof(double) * (pf->n ? pf->n : 1));
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < pf->n; ++i) e[i] = orc_exp((pf->pending ? 0.0 : pf->logw[i]) - M);
    for (int64_t i = 0; i < pf->n; ++i) {
      S += e[i];
      S2 += e[i] * e[i];
    }
    free(e);
  }
  out[0] = M; out[1] = S; out[2] = S2;
}

/* combine per-rank (max, S, S2) in rank order; decision ess < thr */
int orc_combine_stats(const double* st, int R, int64_t n_global, double thr, double* L, double* ess,
                      double* Mout) {
  double M = -INFINITY;
  for (int r = 0; r < R; ++r) if (st[3 * r] > M) M = st[3 * r];
  if (!(M > -INFINITY) || M != M || M == INFINITY) { *L = M; *ess = NAN; *Mout = M; return -1; }
  double S = 0.0, S2 = 0.0;
  for (int r = 0; r < R; ++r) {
    if (!(st[3 * r] > -INFINITY)) continue;
    double e = orc_exp(st[3 * r] - M);
    S += st[3 * r + 1] * e;
    S2 += st[3 * r + 2] * (e * e);
  }
  *L = M + orc_log(S);
  *ess = (S * S) / S2;
  *Mout = M;
  (void)n_global;
  return *ess < thr;
}

uint64_t orc_pf_local_qtotal(orc_pf* pf, double M) {
  int sh = qshift((uint64_t)pf->n_global);
  uint64_t s = 0;
#pragma omp parallel for schedule(static) reduction(+ : s)
  for (int64_t i = 0; i < pf->n; ++i) s += quantize(pf->pending ? 0.0 : pf->logw[i], M, sh);
  return s;
}

/* target of global slot j in [0, S) */
static uint64_t slot_target(const orc_pf* pf, uint64_t S, int64_t j, uint64_t o) {
  if (pf->resampler == ORC_SYSTEMATIC) {
    uint64_t N = (uint64_t)pf->n_global;
    uint64_t Qs = S / N, Rs = S % N;
    return (uint64_t)j * Qs + ((uint64_t)j * Rs + o) / N;
  }
  uint32_t w[4];
  rng(pf->seed, (uint64_t)j, (uint32_t)pf->t, S_RESAMPLE, 0, w);
  return scale_u53(bits53(w[0], w[1]), S);
}

int64_t orc_pf_resample_emit(orc_pf* pf, double M, const uint64_t* totals, int R, int rank,
                             int64_t* slot_out, int64_t* anc_out, double* state_out) {
  int sh = qshift((uint64_t)pf->n_global);
  uint64_t base = 0, S = 0;
  for (int r = 0; r < R; ++r) { if (r < rank) base += totals[r]; S += totals[r]; }
  uint64_t mine = totals[rank];
  /* inclusive local CDF */
  uint64_t* C = malloc(sizeof(uint64_t) * (pf->n ? pf->n : 1));
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < pf->n; ++i) C[i] = quantize(pf->pending ? 0.0 : pf->logw[i], M, sh);
  uint64_t acc = 0;
  for (int64_t i = 0; i < pf->n; ++i) {
    acc += C[i];
    C[i] = acc;
  }
  const double* xs = pf->pending ? pf->anc_state : pf->x;
  uint64_t o = 0;
  if (pf->resampler == ORC_SYSTEMATIC) {
    uint32_t w[4];
    rng(pf->seed, ~0ull, (uint32_t)pf->t, S_RESAMPLE, 0, w);
    o = scale_u53(bits53(w[0], w[1]), S);
  }
  int D = pf->m.d;
  int64_t cnt = 0;
  if (R == 1) {  /* one shard: every slot is this rank's, slot j is emitted j-th */
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < pf->n_global; ++j) {
      uint64_t lt = slot_target(pf, S, j, o);
      int64_t lo = 0, hi = pf->n - 1;
      while (lo < hi) {
        int64_t mid = lo + (hi - lo) / 2;
        if (C[mid] > lt) hi = mid; else lo = mid + 1;
      }
      slot_out[j] = j;
      anc_out[j] = pf->pending ? pf->anc[lo] : pf->lo + lo;
      for (int k = 0; k < D; ++k) state_out[j * D + k] = xs[(size_t)k * pf->n + lo];
    }
    free(C);
    return pf->n_global;
  }
  for (int64_t j = 0; j < pf->n_global; ++j) {
    uint64_t tg = slot_target(pf, S, j, o);
    if (tg < base || tg >= base + mine) continue;
    uint64_t lt = tg - base;
    int64_t lo = 0, hi = pf->n - 1;
    while (lo < hi) {  /* first i with C[i] > lt */
      int64_t mid = lo + (hi - lo) / 2;
      if (C[mid] > lt) hi = mid; else lo = mid + 1;
    }
    slot_out[cnt] = j;
    anc_out[cnt] = pf->pending ? pf->anc[lo] : pf->lo + lo;
    for (int k = 0; k < D; ++k) state_out[cnt * D + k] = xs[(size_t)k * pf->n + lo];
    ++cnt;
  }
  free(C);
  return cnt;
}

void orc_pf_resample_apply(orc_pf* pf, double L, int64_t count, const int64_t* slots,
                           const int64_t* ancs, const double* states) {
  int D = pf->m.d;
  for (int64_t e = 0; e < count; ++e) {
    int64_t i = slots[e] - pf->lo;
    if (i < 0 || i >= pf->n) continue;
    pf->anc[i] = ancs[e];
    for (int k = 0; k < D; ++k) pf->anc_state[(size_t)k * pf->n + i] = states[e * D + k];
  }
  pf->log_ml_est += L - orc_log((double)pf->n_global);
  pf->pending = 1;
  if (pf->cond && pf->n > 0) {  /* the distinguished particle's parent is itself (smc.jl:139) */
    pf->anc[0] = 0;
    for (int k = 0; k < D; ++k) pf->anc_state[(size_t)k * pf->n] = pf->x[(size_t)k * pf->n];
  }
}

int orc_pf_maybe_resample(orc_pf* pf, double thr, double* ess_out) {
  double st[3], L, ess, M;
  orc_pf_local_stats(pf, st);
  int dec = orc_combine_stats(st, 1, pf->n_global, thr, &L, &ess, &M);
  if (ess_out) *ess_out = ess;
  if (dec < 0) return -1;
  if (!dec) return 0;
  uint64_t tot = orc_pf_local_qtotal(pf, M);
  int64_t n = pf->n;
  int D = pf->m.d;
  int64_t* slots = malloc(sizeof(int64_t) * n);
  int64_t* ancs = malloc(sizeof(int64_t) * n);
  double* sts = malloc(sizeof(double) * n * D);
  int64_t c = orc_pf_resample_emit(pf, M, &tot, 1, 0, slots, ancs, sts);
  orc_pf_resample_apply(pf, L, c, slots, ancs, sts);
  free(slots); free(ancs); free(sts);
  return 1;
}

double orc_pf_log_ml_estimate(orc_pf* pf) {
  double st[3], L, ess, M;
  orc_pf_local_stats(pf, st);
  orc_combine_stats(st, 1, pf->n_global, 0.0, &L, &ess, &M);
  return pf->log_ml_est + L - orc_log((double)pf->n_global);
}

void orc_pf_get_log_weights(orc_pf* pf, double* out) {
  for (int64_t i = 0; i < pf->n; ++i) out[i] = pf->pending ? 0.0 : pf->logw[i];
}
void orc_pf_get_state(orc_pf* pf, double* out) {
  double* src = pf->pending ? pf->anc_state : pf->x;
  memcpy(out, src, sizeof(double) * pf->m.d * pf->n);
}
void orc_pf_get_parents(orc_pf* pf, int64_t* out) { memcpy(out, pf->anc, sizeof(int64_t) * pf->n); }
int orc_pf_num_steps(orc_pf* pf) { return pf->t; }

/* The scores of one step's choices under the model (the per-choice score
   fields of src/static_ir/trace.jl:91-129): the latent x_t | x_{t-1} (t = 1:
   the initial distribution) and the observation y_t | x_t; the densities of
   mvnormal.jl:12-16 (forward substitution with the Cholesky factor),
   normal.jl:56-60, categorical.jl:10-12. */
static void model_score(const model_t* m, const obs_t* o, int t, const double* xp, const double* x, double* lat,
                        double* ob) {
  if (m->family == ORC_SLOTS && m->lat == 0) {  /* dense forward substitution (SlotModel::latent_lpdf) */
    int d = m->d;
    const double* L = t == 1 ? m->L0 : m->LQ;
    double u[64], quad = 0.0;
    for (int i = 0; i < d; ++i) {
      double mean;
      if (t == 1) {
        mean = m->mu0[i];
      } else {
        mean = m->uin ? m->b[i] + o->bt[m->snv + i] : m->b[i];
        for (int k = 0; k < d; ++k) mean = fma(m->A[i * d + k], xp[k], mean);
      }
      double r = x[i] - mean;
      for (int k = 0; k < i; ++k) r = fma(-L[i * d + k], u[k], r);
      u[i] = r / L[i * d + i];
      quad = fma(u[i], u[i], quad);
    }
    *lat = (t == 1 ? m->cst0 : m->cstQ) - 0.5 * quad;
  } else if (m->family == ORC_SLOTS && m->lat == 4) {  /* log p(z | z_prev) + mvnormal.jl:12-16 under z */
    const int nz = m->nz, dx = m->d - nz, z = slot_regime(m, x);
    const double* blk = m->SW + z * (2 * dx * dx + dx);
    const double lz = orc_log(t == 1 ? m->prior[z] : m->T[z * nz + slot_regime(m, xp)]);
    const double* L = t == 1 ? m->L0 : blk + dx * dx + dx;
    double u[64], quad = 0.0;
    for (int i = 0; i < dx; ++i) {
      double mean;
      if (t == 1) {
        mean = m->mu0[i];
      } else {
        mean = blk[dx * dx + i];
        for (int k = 0; k < dx; ++k) mean = fma(blk[i * dx + k], xp[k], mean);
      }
      double r = x[i] - mean;
      for (int k = 0; k < i; ++k) r = fma(-L[i * dx + k], u[k], r);
      u[i] = r / L[i * dx + i];
      quad = fma(u[i], u[i], quad);
    }
    *lat = lz + ((t == 1 ? m->cst0 : m->cstQz[z]) - 0.5 * quad);
  } else if (m->family == ORC_SLOTS && m->lat == 3) {  /* categorical.jl:10-12 */
    const int z = slot_onehot(x, m->d);
    *lat = orc_log(t == 1 ? m->prior[z] : m->T[z * m->d + slot_onehot(xp, m->d)]);
  } else if (m->family == ORC_LGSSM) {
    int d = m->d;
    const double* L = t == 1 ? m->L0 : m->LQ;
    double u[64], quad = 0.0;
    for (int i = 0; i < d; ++i) {
      double mean;
      if (t == 1) {
        mean = m->mu0[i];
      } else {
        mean = m->b[i];
        for (int k = 0; k < d; ++k) mean = fma(m->A[i * d + k], xp[k], mean);
      }
      double r = x[i] - mean;
      if (t == 1 || !m->lq_diag)
        for (int k = 0; k < i; ++k) r = fma(-L[i * d + k], u[k], r);
      u[i] = r / L[i * d + i];
      quad = fma(u[i], u[i], quad);
    }
    *lat = (t == 1 ? m->cst0 : m->cstQ) - 0.5 * quad;
  } else if (m->family == ORC_KITAGAWA || m->family == ORC_SLOTS) {
    double mean = m->mu1, inv2 = m->inv2v1, cst = m->cst1;
    if (t > 1) {
      double v = xp[0];
      mean = ((v / 2.0) + 25.0 * (v / (1.0 + v * v))) + o->ct;
      inv2 = m->inv2vx;
      cst = m->cstx;
    }
    double dd = x[0] - mean;
    *lat = -(dd * dd) * inv2 + cst;
  } else if (m->family == ORC_HMM) {
    int z = (int)x[0];
    *lat = orc_log(t == 1 ? m->prior[z] : m->T[z * m->k + (int)xp[0]]);
  } else {
    double ds = x[0] - m->mu_s, di = x[1] - m->mu_i;
    *lat = (-(ds * ds) * m->inv2s + m->csts) + (-(di * di) * m->inv2i + m->csti);
  }
  *ob = model_loglik(m, o, x);
}

/* get_score of every current particle's trace along its genealogy, with the
   per-step latent / observation scores (per_step [t][2][n], nullable) */
/* the trace score columns of every particle under model m and the steps'
   observations obs[0..T) (the filter's own, or rebuilt for other parameters) */
static int scores_with(orc_pf* pf, const model_t* m, const obs_t* obs, double* total, double* per_step) {
  if (pf->t < 1 || (!pf->record_history && pf->t > 1) || pf->lo != 0 || pf->n != pf->n_global) return -1;
  const int T = pf->t, D = pf->m.d;
  const int64_t n = pf->n;
  double* ps = per_step ? per_step : malloc(sizeof(double) * 2 * (size_t)T * (n ? n : 1));
  for (int64_t j = 0; j < n; ++j) {
    int64_t idx = pf->pending ? pf->anc[j] - pf->lo : j;
    double x[64], xp[64];
    const double* cur = pf->record_history ? pf->hx[T - 1] : pf->x;
    for (int k = 0; k < D; ++k) x[k] = cur[(size_t)k * n + idx];
    for (int s = T; s >= 1; --s) {
      int64_t parent = idx;
      if (s > 1) {
        if (pf->hres[s - 1]) parent = pf->hanc[s - 1][idx];
        for (int k = 0; k < D; ++k) xp[k] = pf->hx[s - 2][(size_t)k * n + parent];
      }
      const obs_t* o = &obs[s - 1];
      double lat, ob;
      model_score(m, o, s, xp, x, &lat, &ob);
      ps[((size_t)(s - 1) * 2) * n + j] = lat;
      ps[((size_t)(s - 1) * 2 + 1) * n + j] = ob;
      for (int k = 0; k < D; ++k) x[k] = xp[k];
      idx = parent;
    }
    double tot = 0.0;
    for (int s = 1; s <= T; ++s) tot += ps[((size_t)(s - 1) * 2) * n + j] + ps[((size_t)(s - 1) * 2 + 1) * n + j];
    total[j] = tot;
  }
  if (!per_step) free(ps);
  return 0;
}

int orc_pf_get_scores(orc_pf* pf, double* total, double* per_step) {
  if (pf->t < 1) return -1;
  return scores_with(pf, &pf->m, pf->record_history ? pf->hobs : &pf->obs, total, per_step);
}

/* particle_filter_step!(state, (t, params'...), (UnknownChange(), UnknownChange()...), obs)
   (particle_filter.jl:162-180): the Unfold's parameters change, so its update
   visits every retained kernel application (unfold/generic_update.jl:9-16);
   with no new constraints on them each contributes its new score - old score
   (static_ir/update.jl), then the new application is generated under the new
   parameters.  Here: Delta_j = get_score under the new parameters - under the
   old ones along particle j's trajectory (time-ordered sums), the step under
   the new model, then logw_j += Delta_j.  Same family and dimensions; needs
   the history (one shard). */
int orc_pf_step_params(orc_pf* pf, const double* params, int64_t np, const double* obs, int has_obs, int proposal) {
  if (pf->cond || pf->t < 1 || !pf->record_history || pf->lo != 0 || pf->n != pf->n_global) return -1;
  if (proposal == ORC_PROPOSAL_LINEAR && !pf->m.qlin) return -1;
  model_t m2;
  const model_t* m = &pf->m;
  if (model_build(&m2, m->family, m->d, m->dy, m->k, m->v, params, np)) {
    model_free(&m2);
    return -1;
  }
  if (m->family == ORC_SLOTS) {  /* the same latent form and slot layout (the engine's same_slots) */
    int same = m2.lat == m->lat && m2.K == m->K && m2.uin == m->uin;
    for (int k = 0; same && k < m->K; ++k)
      same = m2.sdist[k] == m->sdist[k] && m2.sm[k] == m->sm[k] && m2.slink[k] == m->slink[k];
    if (!same) {
      model_free(&m2);
      return -1;
    }
  }
  if (proposal != ORC_PROPOSAL_LINEAR && !proposal_ok(&m2, proposal)) {  /* (the linear one: the filter's args) */
    model_free(&m2);
    return -1;
  }
  const int T = pf->t;
  const int64_t n = pf->n;
  obs_t* o2 = malloc(sizeof(obs_t) * (size_t)T);
  for (int s = 1; s <= T; ++s) obs_build(&m2, s, pf->hobs[s - 1].raw, pf->hobs[s - 1].present, &o2[s - 1]);
  double* old_tot = malloc(sizeof(double) * (size_t)(n ? n : 1));
  double* new_tot = malloc(sizeof(double) * (size_t)(n ? n : 1));
  scores_with(pf, &pf->m, pf->hobs, old_tot, NULL);
  scores_with(pf, &m2, o2, new_tot, NULL);
  /* the proposal arguments are the filter's: they carry over */
  memcpy(m2.qa, pf->m.qa, sizeof m2.qa);
  m2.qlin = pf->m.qlin;
  m2.QP = pf->m.QP;
  m2.QL = pf->m.QL;
  m2.cstq = pf->m.cstq;
  memcpy(m2.qu, pf->m.qu, sizeof m2.qu);
  pf->m.QP = pf->m.QL = NULL;
  model_free(&pf->m);
  pf->m = m2;
  memcpy(pf->hobs, o2, sizeof(obs_t) * (size_t)T);
  free(o2);
  int rc = step_impl(pf, obs, has_obs, proposal, NULL);
  if (!rc)
    for (int64_t j = 0; j < n; ++j) pf->logw[j] += new_tot[j] - old_tot[j];
  free(old_tot);
  free(new_tot);
  return rc;
}

/* simulate(model, (T,)) for n traces (static_ir/simulate.jl:23-34, 50-83;
   unfold/simulate.jl): per step the latent is drawn as generate / update draw
   it (particle_init / particle_step, stream S_SIM, no observation), then the
   observation from draw SIM_OBS_DRAW on, scored as a given observation is
   (obs_build + model_loglik); the latent's score is model_score's.  Outputs
   time-major: xs[t][k][n], ys[t][r][n], per_step[t][2][n], total[n]. */
static int simulate_impl(int family, int d, int dy, int k, int v, const double* params, int64_t np, int T,
                         int64_t n, uint64_t seed, const double* inputs, double* xs, double* ys, double* per_step,
                         double* total);
int orc_simulate(int family, int d, int dy, int k, int v, const double* params, int64_t np, int T, int64_t n,
                 uint64_t seed, double* xs, double* ys, double* per_step, double* total) {
  return simulate_impl(family, d, dy, k, v, params, np, T, n, seed, NULL, xs, ys, per_step, total);
}
/* simulate(model, (T, U)) of a slot model with per-step inputs: inputs[T*d],
   row t-1 the input of step t (row 0 unused), as gh_simulate_inputs */
int orc_simulate_inputs(int family, int d, int dy, int k, int v, const double* params, int64_t np, int T, int64_t n,
                        uint64_t seed, const double* inputs, double* xs, double* ys, double* per_step,
                        double* total) {
  if (!inputs) return -1;
  return simulate_impl(family, d, dy, k, v, params, np, T, n, seed, inputs, xs, ys, per_step, total);
}
static int simulate_impl(int family, int d, int dy, int k, int v, const double* params, int64_t np, int T,
                         int64_t n, uint64_t seed, const double* inputs, double* xs, double* ys, double* per_step,
                         double* total) {
  model_t m;
  if (model_build(&m, family, d, dy, k, v, params, np) || T < 1 || (family == ORC_REGRESSION && T != 1) ||
      (family == ORC_SLOTS && (m.uin != (inputs != NULL))) || (family != ORC_SLOTS && inputs)) {
    model_free(&m);  /* (a model with per-step inputs takes them; no other model does) */
    return -1;
  }
  const int D = m.d, DY = (family == ORC_LGSSM || family == ORC_REGRESSION || family == ORC_SLOTS) ? m.dy : 1;
#pragma omp parallel for schedule(static)
  for (int64_t j = 0; j < n; ++j) {
    double x[64], xp[64] = {0}, y[64], z[64];
    double tot = 0.0;
    for (int t = 1; t <= T; ++t) {
      obs_t none, oy;
      double yin[96];
      const int inb = inputs && t > 1;  /* the step's input rides after the dy slot values (bit 4) */
      if (inb) {
        for (int r = 0; r < m.dy; ++r) yin[r] = 0.0;
        for (int i = 0; i < D; ++i) yin[m.dy + i] = inputs[(size_t)(t - 1) * D + i];
        obs_build(&m, t, yin, 16, &none);
      } else {
        obs_build(&m, t, NULL, 0, &none);
      }
      if (t == 1) particle_init(&m, seed, (uint64_t)j, &none, 0, x, S_SIM, 0);
      else particle_step(&m, seed, (uint64_t)j, (uint32_t)t, &none, 0, xp, x, S_SIM, 0);
      if (family == ORC_SLOTS) {
        slot_sim(&m, seed, (uint64_t)j, (uint32_t)t, x, y);
      } else if (family == ORC_LGSSM) {
        normals_at(seed, (uint64_t)j, (uint32_t)t, S_SIM, SIM_OBS_DRAW, DY, z);
        for (int r = 0; r < DY; ++r) {
          double acc = m.c[r];
          for (int q = 0; q < D; ++q) acc = fma(m.H[r * D + q], x[q], acc);
          for (int q = 0; q <= r; ++q) acc = fma(m.LR[r * DY + q], z[q], acc);
          y[r] = acc;
        }
      } else if (family == ORC_HMM) {
        uint32_t w[4];
        rng(seed, (uint64_t)j, (uint32_t)t, S_SIM, SIM_OBS_DRAW, w);
        y[0] = (double)cat_sample(m.E + (int)x[0], m.v, m.k, unif53(w[0], w[1]));
      } else if (family == ORC_KITAGAWA) {
        normals_at(seed, (uint64_t)j, (uint32_t)t, S_SIM, SIM_OBS_DRAW, 1, z);
        y[0] = x[0] * x[0] / 20.0 + m.sy * z[0];
      } else {
        normals_at(seed, (uint64_t)j, (uint32_t)t, S_SIM, SIM_OBS_DRAW, DY, z);
        for (int i = 0; i < DY; ++i) y[i] = (x[0] * m.xs[i] + x[1]) + m.sigma * z[i];
      }
      if (inb) {
        for (int r = 0; r < m.dy; ++r) yin[r] = y[r];
        obs_build(&m, t, yin, ((1 << m.K) - 1) | 16, &oy);
      } else {
        obs_build(&m, t, y, family == ORC_SLOTS ? (1 << m.K) - 1 : 1, &oy);
      }
      double lat, ob;
      model_score(&m, &oy, t, xp, x, &lat, &ob);
      if (xs) for (int q = 0; q < D; ++q) xs[((size_t)(t - 1) * D + q) * n + j] = x[q];
      if (ys) for (int r = 0; r < DY; ++r) ys[((size_t)(t - 1) * DY + r) * n + j] = y[r];
      if (per_step) {
        per_step[((size_t)(t - 1) * 2) * n + j] = lat;
        per_step[((size_t)(t - 1) * 2 + 1) * n + j] = ob;
      }
      tot += lat + ob;
      for (int q = 0; q < D; ++q) xp[q] = x[q];
    }
    if (total) total[j] = tot;
  }
  model_free(&m);
  return 0;
}

int orc_pf_get_history(orc_pf* pf, int t, double* x_out, int32_t* anc_out, int* resampled) {
  if (!pf->record_history || t < 1 || t > pf->t) return -1;
  memcpy(x_out, pf->hx[t - 1], sizeof(double) * pf->m.d * pf->n);
  *resampled = (t >= 2) ? pf->hres[t - 1] : 0;
  if (*resampled && anc_out) memcpy(anc_out, pf->hanc[t - 1], sizeof(int32_t) * pf->n);
  return 0;
}

/* importance_sampling (importance.jl:20-52): generate N times at t=1,
   normalise with logsumexp, lml = L - log N. */
int orc_importance_sampling(int family, int d, int dy, int k, int v, const double* params,
                            int64_t np, const double* obs, int has_obs, int proposal, int64_t n,
                            uint64_t seed, double* lnw, double* states, double* lml) {
  model_t m;
  if (model_build(&m, family, d, dy, k, v, params, np)) { model_free(&m); return -1; }
  obs_t o;
  obs_build(&m, 1, obs, has_obs, &o);
  double x[64];
  double M = -INFINITY;
  for (int64_t i = 0; i < n; ++i) {
    lnw[i] = particle_init(&m, seed, (uint64_t)i, &o, proposal, x, S_INIT, 0);
    for (int kk = 0; kk < m.d; ++kk) states[(size_t)kk * n + i] = x[kk];
    if (lnw[i] > M) M = lnw[i];
  }
  double S = 0.0;
  for (int64_t i = 0; i < n; ++i) S += orc_exp(lnw[i] - M);
  double L = M + orc_log(S);
  for (int64_t i = 0; i < n; ++i) lnw[i] -= L;
  *lml = L - orc_log((double)n);
  model_free(&m);
  return 0;
}

/* ----------------------------------------------------------------- PMMH */
/* Particle-marginal MH over the Kitagawa model (examples/pmmh/example.jl:
   20-79).  The likelihood term is the ParticleFilterCombinator of
   examples/pmmh/pf.jl:14-73: generate/update/regenerate of the :hmm call run a
   particle filter (initialize_particle_filter, then {maybe_resample!;
   particle_filter_step!} for t = 2..T, pf.jl:40-56, with maybe_resample! at
   ESS < N/2 and systematic integer resampling as everywhere here) over the
   model of example.jl:5-22 / model.jl:9-13 (x_1 ~ normal(0, 5); x_t ~
   normal(x_mean(x_{t-1}, t), sqrt(var_x)); y_t ~ normal(x_t^2 / 20,
   sqrt(var_y))) and return its log_ml_estimate as the weight
   (pf.jl:58-73).  do_inference (example.jl:64-79): each iteration applies
   mh(select(:var_x)), mh(select(:var_y)) — regenerate from the normal(0, 2)
   prior, weight = new log-ML - old (mh.jl:14-28) — and the random walks
   mh(tr, var_x_proposal) / var_y_proposal, normal(cur, sqrt(0.5)), weight =
   prior ratio + log-ML ratio, alpha = weight - fwd + bwd (mh.jl:41-62).
   Randomness: move counter u (0 = generate, 1 + 4 iter + m), particle id
   (u << 32) | (chain << 10) | p; the state noise of steps t
   and t + 1 (t even) is one Box-Muller pair drawn at step t.  tests/test_pmmh.py checks
   the inner estimate against the PF oracle (run_pf) on the same model. */
static double pmmh_filter(uint64_t seed, uint64_t c, uint32_t u, double lvx, double lvy, int N,
                          const double* ys, const double* ct, int T, double* x, double* lw, double* xp,
                          uint64_t* C) {
  double var_x = orc_exp(lvx), var_y = orc_exp(lvy);
  double sx = sqrt(var_x), inv2vy = 1.0 / (2.0 * var_y);
  double csty = -0.5 * orc_log(2.0 * 0x1.921fb54442d18p+1 * var_y);
  uint64_t cid = ((uint64_t)u << 32) | (c << 10);
  double logN = orc_log((double)N);
  int shift = qshift((uint64_t)N);
  double z[2];
  for (int p = 0; p < N; ++p) {
    orc_normals(seed, cid | (uint64_t)p, 1, S_INIT, 1, z);
    x[p] = 0.0 + 5.0 * z[0];
    double diff = ys[0] - x[p] * x[p] / 20.0;
    lw[p] = -(diff * diff) * inv2vy + csty;
  }
  double log_ml = 0.0;
  for (int t = 2; t <= T; ++t) {
    double M = -INFINITY, S = 0.0, S2 = 0.0;
    for (int p = 0; p < N; ++p) M = fmax(M, lw[p]);
    for (int p = 0; p < N; ++p) {
      double e = lw[p] > -INFINITY ? orc_exp(lw[p] - M) : 0.0;
      S += e;
      S2 += e * e;
    }
    int fire = (S * S) / S2 < (double)N / 2.0;
    if (fire) {
      log_ml += (M + orc_log(S)) - logN;
      uint64_t acc = 0;
      for (int p = 0; p < N; ++p) { acc += quantize(lw[p], M, shift); C[p] = acc; }
      uint32_t w[4];
      rng(seed, cid, (uint32_t)(t - 1), S_RESAMPLE, 0, w);
      uint64_t o = scale_u53(bits53(w[0], w[1]), acc);
      uint64_t Qs = acc / (uint64_t)N, Rs = acc % (uint64_t)N;
      for (int j = 0; j < N; ++j) {
        uint64_t target = (uint64_t)j * Qs + ((uint64_t)j * Rs + o) / (uint64_t)N;
        int a = 0;
        while (C[a] <= target) ++a;
        xp[j] = x[a];
      }
    } else {
      for (int p = 0; p < N; ++p) xp[p] = x[p];
    }
    for (int p = 0; p < N; ++p) {
      /* steps t and t + 1 (t even) take z0 and z1 of one Box-Muller pair, the
         block of step t (gh_pmmh.h) */
      orc_normals(seed, cid | (uint64_t)p, (uint32_t)(t & ~1), S_STEP, 2, z);
      double v = xp[p];
      double mean = ((v / 2.0) + 25.0 * (v / (1.0 + v * v))) + ct[t - 1];
      x[p] = mean + sx * z[t & 1];
      double diff = ys[t - 1] - x[p] * x[p] / 20.0;
      lw[p] = (fire ? 0.0 : lw[p]) + (-(diff * diff) * inv2vy + csty);
    }
  }
  double M = -INFINITY, S = 0.0;
  for (int p = 0; p < N; ++p) M = fmax(M, lw[p]);
  for (int p = 0; p < N; ++p) S += lw[p] > -INFINITY ? orc_exp(lw[p] - M) : 0.0;
  return log_ml + (M + orc_log(S)) - logN;
}

double orc_pmmh_loglik(uint64_t seed, uint64_t chain, uint32_t u, double lvx, double lvy, int n_inner,
                       const double* ys, int T) {
  if (n_inner < 1 || n_inner > 1024 || T < 1) return NAN;
  double* x = malloc(sizeof(double) * n_inner);
  double* lw = malloc(sizeof(double) * n_inner);
  double* xp = malloc(sizeof(double) * n_inner);
  uint64_t* C = malloc(sizeof(uint64_t) * n_inner);
  double* ct = malloc(sizeof(double) * T);
  for (int t = 1; t <= T; ++t) ct[t - 1] = 8.0 * orc_cos(1.2 * (double)t);
  double ml = pmmh_filter(seed, chain, u, lvx, lvy, n_inner, ys, ct, T, x, lw, xp, C);
  free(x); free(lw); free(xp); free(C); free(ct);
  return ml;
}

int orc_pmmh_run(int64_t chain0, int64_t n_chains, int n_inner, const double* ys, int T, int n_iters,
                 int iter0, uint64_t seed, int init, double* lvx, double* lvy, double* lml, int32_t* accepts,
                 double* hist) {
  if (n_inner < 1 || n_inner > 1024 || T < 1) return 1;
  double* ct = malloc(sizeof(double) * T);
  for (int t = 1; t <= T; ++t) ct[t - 1] = 8.0 * orc_cos(1.2 * (double)t);
  const double sd_rw = 0x1.6a09e667f3bcdp-1;
#pragma omp parallel
  {
  double* x = malloc(sizeof(double) * n_inner);
  double* lw = malloc(sizeof(double) * n_inner);
  double* xp = malloc(sizeof(double) * n_inner);
  uint64_t* C = malloc(sizeof(uint64_t) * n_inner);
#pragma omp for schedule(dynamic, 1)
  for (int64_t cl = 0; cl < n_chains; ++cl) {
    uint64_t c = (uint64_t)(chain0 + cl);
    double vx, vy, ml;
    if (init) {
      double z[2];
      orc_normals(seed, c << 10, 0, S_MH, 2, z);
      vx = 0.0 + 2.0 * z[0];
      vy = 0.0 + 2.0 * z[1];
      ml = pmmh_filter(seed, c, 0, vx, vy, n_inner, ys, ct, T, x, lw, xp, C);
    } else {
      vx = lvx[cl]; vy = lvy[cl]; ml = lml[cl];
    }
    int acc[4] = {0, 0, 0, 0};
    for (int k = 0; k < n_iters; ++k) {
      for (int m = 0; m < 4; ++m) {
        uint32_t u = 1u + 4u * (uint32_t)(iter0 + k) + (uint32_t)m;
        uint64_t cid = ((uint64_t)u << 32) | (c << 10);
        double z[2];
        orc_normals(seed, cid, 0, S_MH, 2, z);
        uint32_t wa[4];
        rng(seed, cid, 0, S_MH, 1, wa);
        double logu = orc_log(unif53(wa[0], wa[1]));
        int on_x = (m & 1) == 0;
        double cur = on_x ? vx : vy, prop, alpha, ml_new;
        if (m < 2) {
          prop = 0.0 + 2.0 * z[0];
          ml_new = pmmh_filter(seed, c, u, on_x ? prop : vx, on_x ? vy : prop, n_inner, ys, ct, T, x, lw, xp, C);
          alpha = ml_new - ml;
        } else {
          prop = cur + sd_rw * z[0];
          ml_new = pmmh_filter(seed, c, u, on_x ? prop : vx, on_x ? vy : prop, n_inner, ys, ct, T, x, lw, xp, C);
          double weight = (orc_normal_logpdf(prop, 0.0, 2.0) - orc_normal_logpdf(cur, 0.0, 2.0)) + (ml_new - ml);
          double fwd = orc_normal_logpdf(prop, cur, sd_rw), bwd = orc_normal_logpdf(cur, prop, sd_rw);
          alpha = (weight - fwd) + bwd;
        }
        if (logu < alpha) {
          if (on_x) vx = prop; else vy = prop;
          ml = ml_new;
          acc[m] += 1;
        }
      }
      if (hist) { hist[(cl * n_iters + k) * 2] = vx; hist[(cl * n_iters + k) * 2 + 1] = vy; }
    }
    lvx[cl] = vx; lvy[cl] = vy; lml[cl] = ml;
    for (int m = 0; m < 4; ++m) accepts[cl * 4 + m] = acc[m];
  }
  free(x); free(lw); free(xp); free(C);
  }
  free(ct);
  return 0;
}

/* ------------------------------------------------------------------ coal */
/* Reversible-jump MH on the coal change-point model (config C3), following
   examples/coal/coal.jl: the model (:47-62) with k ~ poisson(3) change points
   placed by min_uniform_continuous (:18-33), gamma(1, 1/200) rates and the
   piecewise Poisson process of poisson_process.jl:32-51 over the events;
   mcmc_step (:329-336) = rate_move (:103-134), position_move (:140-167) when
   k > 0, birth_death_move (:173-318), each metropolis_hastings with an
   involution (src/inference/mh.jl:85-98; weight = new score - old score +
   bwd score - fwd score + log|J|, trace_translators.jl:848-876), the birth
   Jacobian in closed form |J| = (h_prev + h_next)^2 / h (coal.jl:211-238's
   new_rates differentiated; the reference uses ForwardDiff).

   Score of (k, cp[1..k], h[1..k+1]), b_0 = 0, b_{k+1} = T, c_i the events in
   segment i = (b_{i-1}, b_i] (segment 1 also holds the event at 0):
     logpdf(poisson(3), k) + sum_i logpdf(min_uniform_continuous(cp_{i-1}, T,
     k - i + 1), cp_i) + sum_i logpdf(gamma(1, 1/200), h_i)
     + logpdf(piecewise_poisson_process(b, h), events)
   = k (log 3 - log T) - 3 + sum_i [log 200 - 200 h_i] + sum_i [c_i log h_i - len_i h_i]
   (the order statistics telescope to log k! - k log T; log k! cancels the
   Poisson's).  Moves are scored by their difference (one or two segments).
   tests/test_coal_pins.py checks the score against the reference formulas
   term by term (scipy Poisson / gamma, the min_uniform density, the
   piecewise process) and every move's acceptance ratio against an
   independent Python involution with a finite-difference Jacobian.
   Random numbers: iteration s of chain c uses Philox blocks b = 0..5 of
   (seed, c, s, S_MH, b), two 53-bit uniforms per block; the
   GPU kernel gen_amd/csrc/gh_coal.h computes the same arithmetic. */
#define COAL_KMAX 32
#define COAL_W 68
#define COAL_RATE 200.0
#define COAL_BUCKETS 256

static double coal_u(uint64_t seed, uint64_t c, uint32_t step, uint32_t d) {
  uint32_t w[4];
  rng(seed, c, step, S_MH, d, w);
  return unif53(w[0], w[1]);
}
static double one_minus53(uint32_t a, uint32_t b) {
  uint32_t hi = a >> 11, lo = ((a << 21) & 0xFC000000u) | (b >> 6);
  return fma(-(double)lo, 0x1p-53, fma(-(double)hi, 0x1p-21, 1.0));
}

/* #events <= x (events sorted) */
static int coal_count(const double* ev, int E, double x) {
  int lo = 0, hi = E;
  while (lo < hi) { int mid = (lo + hi) >> 1; if (ev[mid] <= x) lo = mid + 1; else hi = mid; }
  return lo;
}

typedef struct { double T, kb, ktheta, lhalf; const double* ev; int E; } coal_m;
static coal_m coal_model(const double* ev, int E) {
  coal_m m;
  m.T = ev[E - 1];
  m.kb = orc_log(3.0) - orc_log(m.T);
  m.ktheta = orc_log(COAL_RATE);
  m.lhalf = orc_log(0.5);
  m.ev = ev;
  m.E = E;
  return m;
}

/* the score of a row (k, score, cp[32], h[33], pad) from scratch */
static double coal_score(const coal_m* M, const double* row) {
  int k = (int)row[0];
  const double* cp = row + 2;
  const double* h = row + 2 + COAL_KMAX;
  double lower = 0.0;
  for (int i = 0; i < k; ++i) {
    if (!(cp[i] > lower && cp[i] < M->T)) return -INFINITY;
    lower = cp[i];
  }
  for (int i = 0; i <= k; ++i)
    if (!(h[i] > 0.0)) return -INFINITY;
  double sc = (double)k * M->kb - 3.0;
  int n_lo = 0;
  double b_lo = 0.0;
  for (int i = 1; i <= k + 1; ++i) {
    double b_hi = i <= k ? cp[i - 1] : M->T;
    int n_hi = i <= k ? coal_count(M->ev, M->E, b_hi) : M->E;
    double hh = h[i - 1];
    sc += M->ktheta - hh * COAL_RATE;
    sc += (double)(n_hi - n_lo) * orc_log_unit(hh) - (b_hi - b_lo) * hh;
    n_lo = n_hi;
    b_lo = b_hi;
  }
  return sc;
}

static int coal_init(uint64_t seed, uint64_t c, const coal_m* M, double* s) {
  double T = M->T;
  int k = 0, done = 0;
  for (int att = 0; att < 64 && !done; ++att) {
    uint32_t d0 = 100u * (uint32_t)att;
    double u = coal_u(seed, c, 0, d0);
    double p = orc_exp(-3.0), cum = p;
    k = 0;
    while (u >= cum && k < 200) { ++k; p = p * (3.0 / (double)k); cum += p; }
    if (k > COAL_KMAX) continue;
    int ok = 1;
    double lower = 0.0;
    for (int i = 1; i <= k; ++i) {
      double q = coal_u(seed, c, 0, d0 + 1u + (uint32_t)i);
      double m = (double)(k - i + 1);
      double x = T - (T - lower) * orc_exp(orc_log(1.0 - q) / m);
      if (!(x > lower && x < T)) ok = 0;
      s[2 + i - 1] = x;
      lower = x;
    }
    for (int i = 1; i <= k + 1; ++i) {
      double q = coal_u(seed, c, 0, d0 + 40u + (uint32_t)i);
      double x = -orc_log(1.0 - q) / COAL_RATE;
      if (!(x > 0.0)) ok = 0;
      s[2 + COAL_KMAX + i - 1] = x;
    }
    done = ok;
  }
  if (!done) { k = 0; s[2 + COAL_KMAX] = (double)M->E / T; }
  for (int i = k + 1; i <= COAL_KMAX; ++i) s[2 + i - 1] = 0.0;
  for (int i = k + 2; i <= COAL_KMAX + 1; ++i) s[2 + COAL_KMAX + i - 1] = 0.0;
  s[0] = (double)k;
  s[COAL_W - 1] = 0.0;
  s[1] = coal_score(M, s);
  return k;
}

enum { COAL_RATE_MOVE = 0, COAL_POSITION = 1, COAL_BIRTH = 2, COAL_DEATH = 3 };

/* One move's proposal on row s with its uniforms u[] (rate: segment, new rate;
   position: change point, new position; birth: segment, position, u, and
   u1m = 1 - u exactly; death: change point).  Writes the proposed row to out
   (score updated by the difference) and returns alpha (-inf: invalid). */
static double coal_propose(const coal_m* M, const double* s, int move, const double* u, double u1m, double* out) {
  const double T = M->T;
  const double* cp = s + 2;
  const double* h = s + 2 + COAL_KMAX;
  int k = (int)s[0];
  memcpy(out, s, sizeof(double) * COAL_W);
  double* ocp = out + 2;
  double* oh = out + 2 + COAL_KMAX;
  if (move == COAL_RATE_MOVE) {
    int i = (int)(u[0] * (double)(k + 1)) + 1;
    double hh = h[i - 1];
    double lo = hh * 0.5, hi = hh * 2.0;
    double nh = lo + (hi - lo) * u[1];
    double b_lo = i == 1 ? 0.0 : cp[i - 2];
    double b_hi = i == k + 1 ? T : cp[i - 1];
    int n_lo = i == 1 ? 0 : coal_count(M->ev, M->E, b_lo);
    int n_hi = i == k + 1 ? M->E : coal_count(M->ev, M->E, b_hi);
    double dh = nh - hh;
    double delta = ((double)(n_hi - n_lo) * (orc_log_unit(nh) - orc_log_unit(hh)) - (b_hi - b_lo) * dh) - dh * COAL_RATE;
    oh[i - 1] = nh;
    out[1] = s[1] + delta;
    return delta + (orc_log_unit(hi - lo) - orc_log_unit(nh * 2.0 - nh * 0.5));
  }
  if (move == COAL_POSITION) {
    if (k < 1) return -INFINITY;
    int i = (int)(u[0] * (double)k) + 1;
    double lower = i == 1 ? 0.0 : cp[i - 2];
    double upper = i == k ? T : cp[i];
    double x = cp[i - 1];
    double nx = lower + (upper - lower) * u[1];
    if (!(nx > lower && nx < upper)) return -INFINITY;
    double hi_ = h[i - 1], hn = h[i];
    int dc = coal_count(M->ev, M->E, nx) - coal_count(M->ev, M->E, x);
    double delta = (double)dc * (orc_log_unit(hi_) - orc_log_unit(hn)) - (nx - x) * (hi_ - hn);
    ocp[i - 1] = nx;
    out[1] = s[1] + delta;
    return delta;
  }
  if (move == COAL_BIRTH) {
    int i = (int)(u[0] * (double)(k + 1)) + 1;
    double lower = i == 1 ? 0.0 : cp[i - 2];
    double upper = i == k + 1 ? T : cp[i - 1];
    double x = lower + (upper - lower) * u[1];
    double uu = u[2];
    double d_prev = x - lower, d_next = upper - x;
    if (!(k < COAL_KMAX && d_prev > 0.0 && d_next > 0.0 && uu > 0.0)) return -INFINITY;
    double hh = h[i - 1];
    double d_total = d_prev + d_next;
    double lh = orc_log_unit(hh);
    double lr = orc_log_unit(u1m) - orc_log_unit(uu);
    double hp = orc_exp(lh - (d_next / d_total) * lr);
    double hn = orc_exp(lh + (d_prev / d_total) * lr);
    int n_lo = i == 1 ? 0 : coal_count(M->ev, M->E, lower);
    int n_hi = i == k + 1 ? M->E : coal_count(M->ev, M->E, upper);
    int n_x = coal_count(M->ev, M->E, x);
    double lhp = orc_log_unit(hp), lhn = orc_log_unit(hn);
    double delta = ((M->kb + M->ktheta) - ((hp + hn) - hh) * COAL_RATE) +
                   (((double)(n_x - n_lo) * lhp + (double)(n_hi - n_x) * lhn) - (double)(n_hi - n_lo) * lh) -
                   ((d_prev * hp + d_next * hn) - (upper - lower) * hh);
    double fwd = ((k > 0 ? M->lhalf : 0.0) - orc_log_unit((double)(k + 1))) - orc_log_unit(upper - lower);
    double bwd = M->lhalf - orc_log_unit((double)(k + 1));
    double logj = 2.0 * orc_log_unit(hp + hn) - lh;
    /* birth(k, i) (coal.jl:260-283): insert cp at i, rates (hp, hn) at (i, i + 1) */
    for (int j = k; j >= i; --j) ocp[j] = cp[j - 1];
    ocp[i - 1] = x;
    for (int j = k + 1; j >= i + 1; --j) oh[j] = h[j - 1];
    oh[i - 1] = hp;
    oh[i] = hn;
    out[0] = (double)(k + 1);
    out[1] = s[1] + delta;
    return ((delta + bwd) - fwd) + logj;
  }
  /* death */
  if (k < 1) return -INFINITY;
  int i = (int)(u[0] * (double)k) + 1;
  double x = cp[i - 1];
  double lower = i == 1 ? 0.0 : cp[i - 2];
  double upper = i == k ? T : cp[i];
  double d_prev = x - lower, d_next = upper - x;
  if (!(d_prev > 0.0 && d_next > 0.0)) return -INFINITY;
  double hp = h[i - 1], hn = h[i];
  double d_total = d_prev + d_next;
  double lhp = orc_log_unit(hp), lhn = orc_log_unit(hn);
  double hh = orc_exp((d_prev / d_total) * lhp + (d_next / d_total) * lhn);
  double lh = orc_log_unit(hh);
  int n_lo = i == 1 ? 0 : coal_count(M->ev, M->E, lower);
  int n_hi = i == k ? M->E : coal_count(M->ev, M->E, upper);
  int n_x = coal_count(M->ev, M->E, x);
  double delta = (-(M->kb + M->ktheta) - (hh - (hp + hn)) * COAL_RATE) +
                 ((double)(n_hi - n_lo) * lh - ((double)(n_x - n_lo) * lhp + (double)(n_hi - n_x) * lhn)) -
                 ((upper - lower) * hh - (d_prev * hp + d_next * hn));
  double fwd = M->lhalf - orc_log_unit((double)k);
  double bwd = ((k - 1 > 0 ? M->lhalf : 0.0) - orc_log_unit((double)k)) - orc_log_unit(upper - lower);
  double logj = lh - 2.0 * orc_log_unit(hp + hn);
  /* death(k, i) (coal.jl:285-305): remove cp i, rate h at i */
  for (int j = i; j <= k - 1; ++j) ocp[j - 1] = cp[j];
  ocp[k - 1] = 0.0;
  oh[i - 1] = hh;
  for (int j = i + 1; j <= k; ++j) oh[j - 1] = h[j];
  oh[k] = 0.0;
  out[0] = (double)(k - 1);
  out[1] = s[1] + delta;
  return ((delta + bwd) - fwd) + logj;
}

/* sum_i [c_i log h_i - len_i h_i]: the piecewise Poisson process of the row */
static double coal_events_lp(const coal_m* M, const double* row) {
  int k = (int)row[0];
  const double* cp = row + 2;
  const double* h = row + 2 + COAL_KMAX;
  double lp = 0.0, b_lo = 0.0;
  int n_lo = 0;
  for (int i = 1; i <= k + 1; ++i) {
    double b_hi = i <= k ? cp[i - 1] : M->T;
    int n_hi = i <= k ? coal_count(M->ev, M->E, b_hi) : M->E;
    lp += (double)(n_hi - n_lo) * orc_log_unit(h[i - 1]) - (b_hi - b_lo) * h[i - 1];
    n_lo = n_hi;
    b_lo = b_hi;
  }
  return lp;
}

/* mh(trace, select(K)) (coal.jl:338-345; src/dynamic/regenerate.jl): k' by
   inverse CDF from u[0]; the kept change points 1..min(k, k') and rates keep
   their values, change point i > k is drawn by min_uniform_continuous's
   inverse CDF from u[i] (i = 1..32), rate i > k + 1 as gamma(1, 1/200) from
   u[32 + i] (i = 1..33); weight = sum over the kept change points of their
   density under k' minus under k, plus the events' new minus old logpdf.
   Writes the proposed row (score from scratch) and returns the weight
   (-inf: refused or invalid). */
static double coal_regen_k(const coal_m* M, const double* s, const double* u, double* out) {
  const double T = M->T;
  int k = (int)s[0];
  memcpy(out, s, sizeof(double) * COAL_W);
  double p = orc_exp(-3.0), cum = p;
  int kk = 0;
  while (u[0] >= cum && kk < 200) { ++kk; p = p * (3.0 / (double)kk); cum += p; }
  if (kk > COAL_KMAX) return -INFINITY;
  const double* cp = s + 2;
  double* ocp = out + 2;
  double* oh = out + 2 + COAL_KMAX;
  int m = k < kk ? k : kk;
  double dk = (double)(kk - k), w = 0.0, lower = 0.0;
  for (int i = 1; i <= m; ++i) {
    double x = cp[i - 1];
    w += dk * (orc_log_unit(T - x) - orc_log_unit(T - lower)) +
         (orc_log_unit((double)(kk - i + 1)) - orc_log_unit((double)(k - i + 1)));
    lower = x;
  }
  double old_ev = coal_events_lp(M, s);
  int ok = 1;
  for (int i = k + 1; i <= kk; ++i) {
    double mm = (double)(kk - i + 1);
    double x = T - (T - lower) * orc_exp(orc_log(1.0 - u[i]) / mm);
    if (!(x > lower && x < T)) ok = 0;
    ocp[i - 1] = x;
    lower = x;
  }
  for (int i = k + 2; i <= kk + 1; ++i) {
    double x = -orc_log(1.0 - u[32 + i]) / COAL_RATE;
    if (!(x > 0.0)) ok = 0;
    oh[i - 1] = x;
  }
  for (int i = kk + 1; i <= COAL_KMAX; ++i) ocp[i - 1] = 0.0;
  for (int i = kk + 2; i <= COAL_KMAX + 1; ++i) oh[i - 1] = 0.0;
  out[0] = (double)kk;
  if (!ok) return -INFINITY;
  double alpha = w + (coal_events_lp(M, out) - old_ev);
  out[1] = coal_score(M, out);
  return alpha;
}

double orc_coal_regen_k(const double* row, const double* ev, int E, const double* u, double* out) {
  coal_m M = coal_model(ev, E);
  return coal_regen_k(&M, row, u, out);
}

double orc_coal_score(const double* row, const double* ev, int E) {
  coal_m M = coal_model(ev, E);
  return coal_score(&M, row);
}

double orc_coal_propose(const double* row, const double* ev, int E, int move, const double* u, double* out) {
  coal_m M = coal_model(ev, E);
  return coal_propose(&M, row, move, u, 1.0 - u[2], out);
}

int orc_coal_run(int64_t chain0, int64_t n_chains, const double* ev, int E, int n_iters, int iter0,
                 uint64_t seed, int init, double* state, int32_t* accepts, int32_t* khist, int simple) {
  if (E < 1) return 1;
  coal_m M = coal_model(ev, E);
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t cl = 0; cl < n_chains; ++cl) {
    double prop[COAL_W];
    uint64_t c = (uint64_t)(chain0 + cl);
    double* cur = state + cl * COAL_W;
    if (init) {
      memset(cur, 0, sizeof(double) * COAL_W);
      coal_init(seed, c, &M, cur);
    }
    int acc[3] = {0, 0, 0};
    for (int it = 0; it < n_iters; ++it) {
      uint32_t step = (uint32_t)(iter0 + it + 1);
      uint32_t B[6][4];
      for (uint32_t b = 0; b < 6; ++b) rng(seed, c, step, S_MH, b, B[b]);
      double u[3];
      /* rate move */
      u[0] = unif53(B[0][0], B[0][1]);
      u[1] = unif53(B[0][2], B[0][3]);
      double alpha = coal_propose(&M, cur, COAL_RATE_MOVE, u, 0.0, prop);
      if (orc_log_unit(one_minus53(B[1][0], B[1][1])) < alpha) { memcpy(cur, prop, sizeof prop); acc[0]++; }
      /* position move, if k > 0 */
      if ((int)cur[0] > 0) {
        u[0] = unif53(B[1][2], B[1][3]);
        u[1] = unif53(B[2][0], B[2][1]);
        alpha = coal_propose(&M, cur, COAL_POSITION, u, 0.0, prop);
        if (orc_log_unit(one_minus53(B[2][2], B[2][3])) < alpha) { memcpy(cur, prop, sizeof prop); acc[1]++; }
      }
      if (simple) { /* regenerate k (simple_mcmc_step) */
        double ur[66];
        uint32_t w6[4];
        rng(seed, c, step, S_MH, 6u, w6);
        ur[0] = unif53(w6[0], w6[1]);
        int k0 = (int)cur[0];
        for (int i = 1; i <= 32; ++i) ur[i] = i > k0 ? coal_u(seed, c, step, 8u + (uint32_t)i) : 0.0;
        for (int i = 1; i <= 33; ++i) ur[32 + i] = i > k0 + 1 ? coal_u(seed, c, step, 48u + (uint32_t)i) : 0.0;
        alpha = coal_regen_k(&M, cur, ur, prop);
        if (orc_log_unit(one_minus53(w6[2], w6[3])) < alpha) { memcpy(cur, prop, sizeof prop); acc[2]++; }
        if (khist) khist[cl * n_iters + it] = (int32_t)cur[0];
        continue;
      }
      /* birth / death move */
      int k = (int)cur[0];
      int birth = k == 0 || unif53(B[3][0], B[3][1]) < 0.5;
      u[0] = unif53(B[3][2], B[3][3]);
      u[1] = unif53(B[4][0], B[4][1]);
      u[2] = unif53(B[4][2], B[4][3]);
      alpha = coal_propose(&M, cur, birth ? COAL_BIRTH : COAL_DEATH, u, one_minus53(B[4][2], B[4][3]), prop);
      if (orc_log_unit(one_minus53(B[5][0], B[5][1])) < alpha) { memcpy(cur, prop, sizeof prop); acc[2]++; }
      if (khist) khist[cl * n_iters + it] = (int32_t)cur[0];
    }
    for (int m = 0; m < 3; ++m) accepts[cl * 3 + m] = acc[m];
  }
  return 0;
}

/* ------------------------------------------------------ distribution library
   Gen's distributions (src/modeling_library/distributions/) for the batched
   gh_dist_logpdf / gh_dist_random: the logpdf formulas of the reference files
   (file:line at each case) and exact samplers on the Philox stream S_DIST
   keyed (seed, value index, 0, S_DIST | draw) — the specification the engine's
   gen_amd/csrc/gh_dists.h follows operation by operation:
     Box–Muller normals; inversion for the uniforms, bernoulli, categorical,
     exponential, geometric, laplace, cauchy; Marsaglia–Tsang (2000) for gamma
     (boost U^(1/a) below shape 1), inv_gamma = s / G, beta = G1 / (G1 + G2);
     chop-down inversion from the mode for poisson and binomial;
     neg_binomial = poisson(gamma(r, (1-p)/p)) (Distributions.jl's sampler).
   log Gamma is Stirling's series after the recurrence to x >= 8. */
enum { S_DIST = 8 };
enum {
  OD_NORMAL = 1, OD_BNORMAL, OD_MVNORMAL, OD_UNIF, OD_UDISC, OD_BERN, OD_CAT, OD_GAMMA, OD_INVGAMMA, OD_BETA,
  OD_EXP, OD_POIS, OD_BINOM, OD_NEGBINOM, OD_GEOM, OD_LAPLACE, OD_CAUCHY, OD_PWUNIF, OD_BETAUNIF
};
#define OD_PI 0x1.921fb54442d18p+1
#define OD_GAMMA_ITERS 60
#define OD_GAMMA_BOOST 120u
#define OD_SECOND 128u
#define OD_CHOP_MAX (1 << 24)

double orc_log1p(double y) {
  double u = 1.0 + y;
  if (u == 1.0) return y;
  if (u == 0.0) return -INFINITY;
  return orc_log(u) - ((u - 1.0) - y) / u;
}

/* log Gamma(x) = Stirling (x - 1/2) log x - x + log sqrt(2 pi) + sum B_2k / (2k (2k-1) x^(2k-1)) */
double orc_lgamma(double x) {
  if (x != x) return x;
  if (x <= 0.0) return x == 0.0 ? INFINITY : NAN;
  if (x == INFINITY) return x;
  double prod = 1.0;
  while (x < 8.0) { prod *= x; x += 1.0; }
  double r = 1.0 / x, r2 = r * r;
  static const double B[7] = {1.0 / 12.0, -1.0 / 360.0, 1.0 / 1260.0, -1.0 / 1680.0, 1.0 / 1188.0,
                              -691.0 / 360360.0, 1.0 / 156.0};
  double s = B[6];
  for (int k = 5; k >= 0; --k) s = fma(s, r2, B[k]);
  double st = ((x - 0.5) * orc_log(x) - x) + (0x1.d67f1c864beb5p-1 + s * r);
  return prod == 1.0 ? st : st - orc_log(prod);
}

static double od_xlogy(double x, double y) { return x == 0.0 ? 0.0 : x * orc_log(y); }
static double od_xlog1py(double x, double y) { return x == 0.0 ? 0.0 : x * orc_log1p(y); }

static void od_block(const od_rng* r, uint32_t draw, uint32_t w[4]) { rng(r->seed, r->id, r->t, r->stream, r->base + draw, w); }
static double od_u(const od_rng* r, uint32_t draw) {
  uint32_t w[4];
  od_block(r, draw, w);
  return unif53(w[0], w[1]);
}
static double od_one_minus_u(uint32_t a, uint32_t b) {
  uint32_t hi = a >> 11, lo = ((a << 21) & 0xFC000000u) | (b >> 6);
  return fma(-(double)lo, 0x1p-53, fma(-(double)hi, 0x1p-21, 1.0));
}
static double od_upos(const od_rng* r, uint32_t draw) {
  uint32_t w[4];
  od_block(r, draw, w);
  return od_one_minus_u(w[0], w[1]);
}
static double od_normal(const od_rng* r, uint32_t draw) {
  uint32_t w[4];
  od_block(r, draw, w);
  double z0, z1;
  box_muller(w[0], w[1], w[2], &z0, &z1);
  return z0;
}
static int od_cat(const double* p, int K, double u) {
  double total = 0.0;
  for (int k = 0; k < K; ++k) total += p[k];
  double target = u * total, cum = 0.0;
  int last = -1;
  for (int k = 0; k < K; ++k) {
    cum += p[k];
    if (p[k] > 0.0) last = k;
    if (cum > target && p[k] > 0.0) return k;
  }
  return last;
}

/* Gamma(a, 1): Marsaglia & Tsang, "A simple method for generating gamma
   variables" (2000); round i: normal from draw d0 + 2i, uniform from d0 + 2i + 1 */
static double od_gamma(const od_rng* r, double a, uint32_t d0) {
  if (!(a > 0.0)) return NAN;
  double boost = 1.0;
  if (a < 1.0) {
    boost = orc_exp(orc_log(od_upos(r, d0 + OD_GAMMA_BOOST)) / a);
    a = a + 1.0;
  }
  double d = a - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d);
  for (int i = 0; i < OD_GAMMA_ITERS; ++i) {
    double x = od_normal(r, d0 + 2u * (uint32_t)i);
    double v = 1.0 + c * x;
    if (v <= 0.0) continue;
    v = v * v * v;
    double u = od_upos(r, d0 + 2u * (uint32_t)i + 1u);
    double x2 = x * x;
    if (u < 1.0 - 0.0331 * (x2 * x2)) return (d * v) * boost;
    if (orc_log(u) < 0.5 * x2 + d * ((1.0 - v) + orc_log(v))) return (d * v) * boost;
  }
  return NAN;
}

/* chop-down inversion from the mode: U - pmf(m) - pmf(m+1) - pmf(m-1) - ... */
static double od_poisson(const od_rng* r, double lam, uint32_t draw) {
  if (lam == 0.0) return 0.0;
  if (!(lam > 0.0) || lam == INFINITY) return NAN;
  double m = floor(lam), u = od_u(r, draw);
  double pm = orc_exp(od_xlogy(m, lam) - lam - orc_lgamma(m + 1.0));
  u -= pm;
  if (u <= 0.0) return m;
  double lo = m, hi = m, pl = pm, ph = pm;
  for (int it = 0; it < OD_CHOP_MAX; ++it) {
    hi += 1.0; ph = ph * lam / hi; u -= ph;
    if (u <= 0.0) return hi;
    if (lo > 0.0) { pl = pl * lo / lam; lo -= 1.0; u -= pl; if (u <= 0.0) return lo; }
    if (ph == 0.0 && (lo <= 0.0 || pl == 0.0)) break;
  }
  return m;
}

static double od_binomial(const od_rng* r, double n, double p, uint32_t draw) {
  if (!(p >= 0.0 && p <= 1.0) || !(n >= 0.0)) return NAN;
  if (p == 0.0 || n == 0.0) return 0.0;
  if (p == 1.0) return n;
  double q = 1.0 - p, m = floor((n + 1.0) * p);
  if (m > n) m = n;
  double u = od_u(r, draw);
  double pm = orc_exp(((orc_lgamma(n + 1.0) - orc_lgamma(m + 1.0)) - orc_lgamma(n - m + 1.0)) + od_xlogy(m, p) +
                      od_xlog1py(n - m, -p));
  u -= pm;
  if (u <= 0.0) return m;
  double pq = p / q, qp = q / p, lo = m, hi = m, pl = pm, ph = pm;
  for (int it = 0; it < OD_CHOP_MAX; ++it) {
    if (hi < n) { ph = ph * ((n - hi) / (hi + 1.0)) * pq; hi += 1.0; u -= ph; if (u <= 0.0) return hi; }
    if (lo > 0.0) { pl = pl * (lo / (n - lo + 1.0)) * qp; lo -= 1.0; u -= pl; if (u <= 0.0) return lo; }
    if ((hi >= n || ph == 0.0) && (lo <= 0.0 || pl == 0.0)) break;
  }
  return m;
}

static double od_beta_lp(double v, double a, double b) { /* beta.jl:13-16 */
  if (v < 0.0 || v > 1.0) return -INFINITY;
  double lb = (orc_lgamma(a) + orc_lgamma(b)) - orc_lgamma(a + b);
  return ((a - 1.0) * orc_log(v) + (b - 1.0) * orc_log1p(-v)) - lb;
}

/* row P of one value; x[k * xs] its components; mvnormal's row is derived: mu | L | cst */
static double od_logpdf(int dist, const double* x, int64_t xs, const double* P, int D, int K) {
  double v = x[0];
  switch (dist) {
    case OD_NORMAL: { /* normal.jl:56-60 */
      double var = P[1] * P[1], diff = v - P[0];
      return -(diff * diff) / (2.0 * var) - 0.5 * orc_log(2.0 * OD_PI * var);
    }
    case OD_BNORMAL: { /* normal.jl:62-71: sum of the elementwise logpdfs */
      double s = 0.0;
      for (int k = 0; k < D; ++k) {
        double var = P[D + k] * P[D + k], diff = x[k * xs] - P[k];
        s += -(diff * diff) / (2.0 * var) - 0.5 * orc_log(2.0 * OD_PI * var);
      }
      return s;
    }
    case OD_MVNORMAL: { /* mvnormal.jl:12-16 */
      const double* L = P + D;
      double u[32], quad = 0.0;
      for (int i = 0; i < D; ++i) {
        double r = x[i * xs] - P[i];
        for (int k = 0; k < i; ++k) r = fma(-L[i * D + k], u[k], r);
        u[i] = r / L[i * D + i];
        quad = fma(u[i], u[i], quad);
      }
      return P[D + D * D] - 0.5 * quad;
    }
    case OD_UNIF: return (v >= P[0] && v <= P[1]) ? -orc_log(P[1] - P[0]) : -INFINITY; /* uniform_continuous.jl:12-14 */
    case OD_UDISC: return (v >= P[0] && v <= P[1] && v == floor(v)) ? -orc_log((P[1] - P[0]) + 1.0) : -INFINITY;
    case OD_BERN: return v != 0.0 ? orc_log(P[0]) : orc_log(1.0 - P[0]); /* bernoulli.jl:10-12 */
    case OD_CAT: return (v > 0.0 && v <= (double)K && v == floor(v)) ? orc_log(P[(int)v - 1]) : -INFINITY;
    case OD_GAMMA: /* gamma.jl:10-16 */
      return v > 0.0 ? (((P[0] - 1.0) * orc_log(v) - (v / P[1])) - P[0] * orc_log(P[1])) - orc_lgamma(P[0]) : -INFINITY;
    case OD_INVGAMMA: /* inv_gamma.jl:12-18 */
      return v > 0.0 ? ((P[0] * orc_log(P[1]) - (P[0] + 1.0) * orc_log(v)) - orc_lgamma(P[0])) - (P[1] / v) : -INFINITY;
    case OD_BETA: return od_beta_lp(v, P[0], P[1]);
    case OD_EXP: { double sc = 1.0 / P[0]; return v < 0.0 ? -INFINITY : -orc_log(sc) - v / sc; } /* exponential.jl:10-13 */
    case OD_POIS: return v < 0.0 ? -INFINITY : (v * orc_log(P[0]) - P[0]) - orc_lgamma(v + 1.0); /* poisson.jl:10-12 */
    case OD_BINOM:
      if (v < 0.0 || v > P[0] || v != floor(v)) return -INFINITY;
      return (((orc_lgamma(P[0] + 1.0) - orc_lgamma(v + 1.0)) - orc_lgamma(P[0] - v + 1.0)) + od_xlogy(v, P[1])) +
             od_xlog1py(P[0] - v, -P[1]);
    case OD_NEGBINOM:
      if (v < 0.0 || v != floor(v)) return -INFINITY;
      return (((orc_lgamma(v + P[0]) - orc_lgamma(P[0])) - orc_lgamma(v + 1.0)) + od_xlogy(P[0], P[1])) +
             od_xlog1py(v, -P[1]);
    case OD_GEOM:
      if (v < 0.0 || v != floor(v)) return -INFINITY;
      return orc_log(P[0]) + od_xlog1py(v, -P[0]);
    case OD_LAPLACE: return -fabs(v - P[0]) / P[1] - orc_log(2.0 * P[1]); /* laplace.jl:10-13 */
    case OD_CAUCHY: { double z = (v - P[0]) / P[1]; return -(orc_log(OD_PI * P[1]) + orc_log1p(z * z)); }
    case OD_PWUNIF: { /* piecewise_uniform.jl:30-43 */
      if (v <= P[0] || v >= P[K]) return -INFINITY;
      int bin = 0;
      while (v > P[bin + 1]) ++bin;
      return orc_log(P[K + 1 + bin]) - orc_log(P[bin + 1] - P[bin]);
    }
    default: { /* beta_uniform.jl:12-20 */
      if (v < 0.0 || v > 1.0) return -INFINITY;
      double lbeta = orc_log(P[0]) + od_beta_lp(v, P[1], P[2]), lunif = orc_log(1.0 - P[0]);
      double m = lbeta > lunif ? lbeta : lunif;
      if (m == -INFINITY) return m;
      return m + orc_log(orc_exp(lbeta - m) + orc_exp(lunif - m));
    }
  }
}

static void od_random(int dist, const od_rng* r, double* x, int64_t xs, const double* P, int D, int K) {
  const uint64_t seed = r->seed, id = r->id;  /* (the vector draws: distribution entry points only) */
  switch (dist) {
    case OD_NORMAL: x[0] = P[0] + P[1] * od_normal(r, 0); return; /* normal.jl:96 */
    case OD_BNORMAL:
    case OD_MVNORMAL: {
      double z[32];
      normals_at(seed, id, 0, S_DIST, 0, D, z);
      if (dist == OD_BNORMAL) {
        for (int k = 0; k < D; ++k) x[k * xs] = P[k] + P[D + k] * z[k];
      } else {
        const double* L = P + D;
        for (int i = 0; i < D; ++i) {
          double acc = P[i];
          for (int k = 0; k <= i; ++k) acc = fma(L[i * D + k], z[k], acc);
          x[i * xs] = acc;
        }
      }
      return;
    }
    case OD_UNIF: x[0] = od_u(r, 0) * (P[1] - P[0]) + P[0]; return; /* uniform_continuous.jl:21-23 */
    case OD_UDISC: x[0] = P[0] + floor(od_u(r, 0) * ((P[1] - P[0]) + 1.0)); return;
    case OD_BERN: x[0] = od_u(r, 0) < P[0] ? 1.0 : 0.0; return; /* bernoulli.jl:19 */
    case OD_CAT: x[0] = (double)(od_cat(P, K, od_u(r, 0)) + 1); return;
    case OD_GAMMA: x[0] = P[1] * od_gamma(r, P[0], 0); return;
    case OD_INVGAMMA: x[0] = P[1] / od_gamma(r, P[0], 0); return;
    case OD_BETA: {
      double g1 = od_gamma(r, P[0], 0), g2 = od_gamma(r, P[1], OD_SECOND);
      x[0] = g1 / (g1 + g2);
      return;
    }
    case OD_EXP: x[0] = (1.0 / P[0]) * -orc_log(od_upos(r, 0)); return;
    case OD_POIS: x[0] = od_poisson(r, P[0], 0); return;
    case OD_BINOM: x[0] = od_binomial(r, P[0], P[1], 0); return;
    case OD_NEGBINOM: {
      double lam = ((1.0 - P[1]) / P[1]) * od_gamma(r, P[0], 0);
      x[0] = od_poisson(r, lam, OD_SECOND);
      return;
    }
    case OD_GEOM: x[0] = floor(orc_log(od_upos(r, 0)) / orc_log1p(-P[0])) + 0.0; return;
    case OD_LAPLACE: {
      uint32_t w[4];
      od_block(r, 0, w);
      double e = -orc_log(od_one_minus_u(w[0], w[1]));
      x[0] = P[0] + P[1] * ((w[2] & 1u) ? -e : e);
      return;
    }
    case OD_CAUCHY: {
      uint32_t w[4];
      od_block(r, 0, w);
      double u = ((double)bits53(w[0], w[1]) + 0.5) * 0x1p-53, s, c;
      orc_sincos_2pi(u * 0.5, &s, &c);
      x[0] = P[0] - P[1] * (c / s);
      return;
    }
    case OD_PWUNIF: {
      int bin = od_cat(P + K + 1, K, od_u(r, 0));
      x[0] = od_u(r, 1) * (P[bin + 1] - P[bin]) + P[bin];
      return;
    }
    default: /* beta_uniform.jl:36-42 */
      if (od_u(r, 255) < P[0]) {
        double g1 = od_gamma(r, P[1], 0), g2 = od_gamma(r, P[2], OD_SECOND);
        x[0] = g1 / (g1 + g2);
      } else {
        x[0] = od_u(r, 254);
      }
  }
}

/* the parameter row layout of gh_dist_desc; returns the derived row length or -1 */
static int od_row(int dist, int dim, int np, const double* params, double* row, int* D, int* K) {
  *D = 1; *K = 0;
  if (dist == OD_BNORMAL) { *D = dim; }
  if (dist == OD_CAT) *K = np;
  if (dist == OD_PWUNIF) *K = (np - 1) / 2;
  if (dist == OD_MVNORMAL) {
    int d = dim;
    *D = d;
    memset(row, 0, sizeof(double) * (d + d * d + 1));
    memcpy(row, params, sizeof(double) * d);
    if (chol(d, params + d, row + d)) return -1;
    row[d + d * d] = gauss_cst(d, row + d);
    return d + d * d + 1;
  }
  memcpy(row, params, sizeof(double) * np);
  return np;
}

int orc_dist_logpdf(int dist, int dim, int np, int stride, const double* params, int64_t n, const double* x,
                    double* out) {
  double row[32 + 32 * 32 + 1];
  int D, K;
  if (np > 1024 + 33) return -1;
  for (int64_t i = 0; i < n; ++i) {
    if (i == 0 || stride) if (od_row(dist, dim, np, params + i * stride, row, &D, &K) < 0) return -1;
    out[i] = od_logpdf(dist, x + i, n, row, D, K);
  }
  return 0;
}

int orc_dist_random(int dist, int dim, int np, int stride, const double* params, int64_t n, uint64_t seed,
                    double* out) {
  double row[32 + 32 * 32 + 1];
  int D, K;
  if (np > 1024 + 33) return -1;
  for (int64_t i = 0; i < n; ++i) {
    if (i == 0 || stride) if (od_row(dist, dim, np, params + i * stride, row, &D, &K) < 0) return -1;
    const od_rng r = {seed, (uint64_t)i, 0, S_DIST, 0};
    od_random(dist, &r, out + i, n, row, D, K);
  }
  return 0;
}
