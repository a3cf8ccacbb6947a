// Host-side sanitizer run ("Race detection"): every C ABI of
// cpp_ls_lib.so called from a native program, with the library's HOST code
// and this driver built under -fsanitize=address,undefined (device code is
// not instrumented: GPU ASan is not available on this pool).  Exercises the
// allocation / staging / error paths of the engine, the reference ABI, the
// serving, preparation and similar-movies contexts, with small inputs, and
// checks return codes and finiteness (numerical parity is the job of tests/).
//
// Build: make -C tools/asan      Run (GPU box): tools/asan/run.sh
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "cpp_ls_lib.h"
#include "mr_als.h"
#include "mr_prep.h"
#include "mr_serving.h"
#include "mr_similar.h"

static int g_fail = 0;
#define EXPECT(cond, what)                                                   \
  do {                                                                       \
    if (!(cond)) {                                                           \
      fprintf(stderr, "FAIL %s:%d %s (%s)\n", __FILE__, __LINE__, what,      \
              mr_last_error());                                              \
      ++g_fail;                                                              \
    }                                                                        \
  } while (0)

static bool finite_all(const std::vector<double>& v) {
  for (double x : v)
    if (!std::isfinite(x)) return false;
  return true;
}

struct Ratings {
  std::vector<int> u, i;
  std::vector<double> r;
};

// every user rates ~density of the items, at least k+1; every item >= k
static Ratings make_ratings(int nu, int ni, int k, double density, unsigned seed) {
  std::mt19937 g(seed);
  std::uniform_real_distribution<double> U01(0.0, 1.0);
  Ratings R;
  for (int a = 0; a < nu; ++a)
    for (int b = 0; b < ni; ++b)
      if (U01(g) < density || (b + a) % ni < k + 1) {
        R.u.push_back(a);
        R.i.push_back(b);
        R.r.push_back(0.5 * (1 + (int)(U01(g) * 10)) - 2.75);
      }
  return R;
}

static void run_reference_abi() {
  const int k = 8, nu = 60, ni = 50;
  Ratings R = make_ratings(nu, ni, k, 0.4, 1);
  std::mt19937 g(2);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  std::vector<double> Uf(nu * (k + 1)), Vf(ni * k);
  for (auto& x : Uf) x = U(g);
  for (auto& x : Vf) x = U(g);
  set_thread_count(12345);
  EXPECT(get_thread_count() == 12345, "thread count round trip");
  const int ret = als_from_python(R.u.data(), R.i.data(), (int)R.r.size(), R.r.data(), k,
                                  (int)Uf.size(), Uf.data(), (int)Vf.size(), Vf.data(), 0.01, 5, 1);
  EXPECT(ret >= 0 && finite_all(Uf) && finite_all(Vf), "als_from_python");
  // wrong factor length -> error, caller buffers untouched
  std::vector<double> Ubad(5, 7.0);
  EXPECT(als_from_python(R.u.data(), R.i.data(), (int)R.r.size(), R.r.data(), k, 5, Ubad.data(),
                         (int)Vf.size(), Vf.data(), 0.01, 5, 1) < 0,
         "als_from_python rejects a short factor table");
  // general CSR CG (both variants)
  const int rows = 200, cols = 50;
  std::vector<int> rp(1, 0), ci;
  std::vector<double> v, b(rows), x(cols, 0.0);
  for (int r = 0; r < rows; ++r) {
    for (int c = 0; c < cols; ++c)
      if ((r * 7 + c * 3) % 5 == 0) {
        ci.push_back(c);
        v.push_back(U(g));
      }
    rp.push_back((int)ci.size());
    b[r] = U(g);
  }
  double rr = -1.0;
  int it = cg_least_squares_from_python(rows, cols, rp.data(), ci.data(), v.data(), rows, b.data(),
                                        cols, x.data(), 0.01, 100, &rr);
  EXPECT(it >= 0 && rr >= 0.0 && finite_all(x), "cg_least_squares_from_python");
  std::fill(x.begin(), x.end(), 0.0);
  it = cg_least_squares2_from_python(rows, cols, rp.data(), ci.data(), v.data(), rows, b.data(),
                                     cols, x.data(), 0.01, 100, nullptr);
  EXPECT(it >= 0 && finite_all(x), "cg_least_squares2_from_python");
  std::vector<int> cbad = ci;
  cbad[3] = cols + 4;
  EXPECT(cg_least_squares_from_python(rows, cols, rp.data(), cbad.data(), v.data(), rows,
                                      b.data(), cols, x.data(), 0.01, 100, nullptr) < 0,
         "cg rejects an out-of-range column");
}

static void run_engine(int k, int chunk) {
  const int nu = 300, ni = 200;
  Ratings R = make_ratings(nu, ni, k, 0.6, 3 + k);
  mr_set_gram_chunk(chunk);
  mr_als* ctx = mr_als_create(0, k, nu, ni, (long long)R.r.size(), R.u.data(), R.i.data(),
                              R.r.data());
  EXPECT(ctx, "mr_als_create");
  if (!ctx) return;
  std::mt19937 g(4);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  std::vector<double> Uf(nu * (k + 1)), Vf(ni * k), U2(Uf.size()), V2(Vf.size());
  for (auto& x : Uf) x = U(g);
  for (auto& x : Vf) x = U(g);
  EXPECT(mr_als_set_factors(ctx, Uf.data(), Vf.data()) == 0, "set_factors");
  EXPECT(mr_als_set_timing(ctx, 1) == 0, "set_timing");
  for (int opt : {0, 1})
    EXPECT(mr_als_set_option(ctx, MR_OPT_CG_SPECULATE, opt * 2) == 0, "speculate option");
  EXPECT(mr_als_run(ctx, 0.01, 4) >= 0, "mr_als_run");
  EXPECT(mr_als_set_option(ctx, MR_OPT_FUSE_START, 0) == 0, "fuse option");
  EXPECT(mr_als_iterate(ctx, 2) == 0, "mr_als_iterate");
  double frr = 0.0;
  EXPECT(mr_als_half_step(ctx, MR_SIDE_ITEMS, &frr) >= 0, "half_step");
  EXPECT(mr_als_get_factors(ctx, U2.data(), V2.data()) == 0 && finite_all(U2) && finite_all(V2),
         "get_factors");
  mr_stats st;
  EXPECT(mr_als_get_stats(ctx, &st) == 0 && st.iterations >= 3, "get_stats");
  EXPECT(mr_als_reset_stats(ctx) == 0, "reset_stats");
  const int K = k + 1;
  std::vector<int> ents = {0, nu / 2, nu - 1};
  std::vector<double> G(ents.size() * K * K), c(ents.size() * K);
  EXPECT(mr_als_get_normal_equations(ctx, MR_SIDE_USERS, (int)ents.size(), ents.data(), G.data(),
                                     c.data()) == 0 && finite_all(G),
         "get_normal_equations");
  std::vector<double> r(nu * K), p(nu * K), q(nu * K);
  EXPECT(mr_als_get_cg_vectors(ctx, MR_SIDE_USERS, r.data(), p.data(), q.data()) == 0,
         "get_cg_vectors");
  const long long nw = mr_als_work_items(ctx, MR_SIDE_ITEMS);
  std::vector<long long> off(ni + 1), wb(nw);
  std::vector<int> idx(R.r.size()), wl(nw), we(nw), ws(nw);
  std::vector<float> val(R.r.size());
  EXPECT(mr_als_get_layout(ctx, MR_SIDE_ITEMS, off.data(), idx.data(), val.data(), wb.data(),
                           wl.data(), we.data(), ws.data()) == 0 && off[ni] == (long long)R.r.size(),
         "get_layout");
  std::vector<double> pred(R.r.size());
  EXPECT(mr_als_predict(ctx, (long long)R.r.size(), R.u.data(), R.i.data(), pred.data()) == 0 &&
             finite_all(pred),
         "predict");
  std::vector<int> bad = {0, nu + 3};
  EXPECT(mr_als_predict(ctx, 2, bad.data(), bad.data(), pred.data()) < 0, "predict rejects ids");
  EXPECT(mr_als_set_solver(ctx, MR_SOLVER_CHOLESKY, 1e-3) == 0 && mr_als_iterate(ctx, 1) == 0,
         "cholesky iterate");
  EXPECT(mr_als_init_factors(ctx, 7) == 0, "init_factors");
  mr_als_destroy(ctx);
  // an out-of-range id fails cleanly
  std::vector<int> ubad = R.u;
  ubad[ubad.size() / 2] = nu + 1;
  mr_als* c2 = mr_als_create(0, k, nu, ni, (long long)R.r.size(), ubad.data(), R.i.data(),
                             R.r.data());
  EXPECT(!c2, "mr_als_create rejects an out-of-range user id");
  if (c2) mr_als_destroy(c2);
  mr_set_gram_chunk(2048);
}

static void run_serving() {
  const int k = 11, n_als = 400, n_users = 30;
  std::mt19937 g(5);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  std::vector<double> F(n_als * k);
  for (auto& x : F) x = U(g);
  std::vector<int> cand_als, cand_mid;
  std::vector<double> cand_med;
  for (int j = 0; j < n_als; j += 1) {
    cand_als.push_back(j);
    cand_mid.push_back(1000 + 3 * j);
    cand_med.push_back(3.0 + 0.5 * (j % 3));
  }
  mr_rec* rec = mr_rec_create(0, k, n_als, F.data(), (int)cand_als.size(), cand_als.data(),
                              cand_mid.data(), cand_med.data());
  EXPECT(rec && mr_rec_num_candidates(rec) == n_als, "mr_rec_create");
  if (!rec) return;
  std::vector<long long> off(1, 0);
  std::vector<int> ai;
  std::vector<double> rt;
  for (int u = 0; u < n_users; ++u) {
    for (int t = 0; t < k + 5 + u; ++t) {
      ai.push_back((u * 37 + t * 11) % n_als);
      rt.push_back(0.5 * (1 + (t * 7 + u) % 10));
    }
    off.push_back((long long)ai.size());
  }
  std::vector<double> x(n_users * (k + 1));
  std::vector<int> method(n_users);
  EXPECT(mr_rec_fold_in(rec, n_users, off.data(), ai.data(), rt.data(), x.data(), method.data()) ==
             0 && finite_all(x),
         "fold_in");
  std::vector<double> sc((size_t)n_users * n_als);
  EXPECT(mr_rec_scores(rec, n_users, x.data(), sc.data()) == 0 && finite_all(sc), "scores");
  const int nr = 20;
  std::vector<long long> eo(n_users + 1);
  std::vector<int> ec;
  for (int u = 0; u < n_users; ++u) {
    eo[u] = (long long)ec.size();
    for (long long j = off[u]; j < off[u + 1]; ++j) ec.push_back(ai[j]);
  }
  eo[n_users] = (long long)ec.size();
  std::vector<int> omid(n_users * nr), ocnt(n_users);
  std::vector<double> osc(n_users * nr);
  EXPECT(mr_rec_top_n(rec, n_users, x.data(), eo.data(), ec.data(), nr, omid.data(), osc.data(),
                      ocnt.data()) == 0,
         "top_n");
  EXPECT(mr_rec_top_n(rec, n_users, x.data(), nullptr, nullptr, 5000, omid.data(), osc.data(),
                      ocnt.data()) < 0,
         "top_n rejects num_results > 1024");
  std::vector<int> urow(n_users), cnd(ai.size());
  for (int u = 0; u < n_users; ++u) urow[u] = u;
  for (size_t j = 0; j < ai.size(); ++j) cnd[j] = (j % 9 == 0) ? -1 : ai[j];
  std::vector<double> agr(n_users), pr(ai.size());
  std::vector<long long> na(n_users), nd(n_users);
  std::vector<double> sse(n_users);          // per test user (mr_serving.h)
  std::vector<long long> npred(n_users);
  EXPECT(mr_rec_evaluate(rec, n_users, x.data(), n_users, urow.data(), off.data(), cnd.data(),
                         rt.data(), agr.data(), na.data(), nd.data(), pr.data(), sse.data(),
                         npred.data()) == 0,
         "evaluate");
  EXPECT(mr_rank_agreement(0, n_users, off.data(), rt.data(), pr.data(), agr.data(), na.data(),
                           nd.data()) == 0,
         "rank_agreement");
  double ms[6];
  EXPECT(mr_rec_last_kernel_ms(rec, ms) == 0, "last_kernel_ms");
  mr_rec_destroy(rec);
}

static void run_prep() {
  const long long n = 20000;
  std::mt19937 g(6);
  std::vector<int> u(n), m(n);
  std::vector<double> r(n);
  for (long long j = 0; j < n; ++j) {
    u[j] = (int)(g() % 700) * 3;
    m[j] = (int)(g() % 300) * 5 + 1;
    r[j] = 0.5 * (1 + g() % 10);
  }
  mr_prep* p = mr_prep_create(0, n, u.data(), m.data(), r.data());
  EXPECT(p, "mr_prep_create");
  if (!p) return;
  int ub = 0, mb = 0;
  EXPECT(mr_prep_id_bounds(p, &ub, &mb) == 0 && ub > 0 && mb > 0, "id_bounds");
  std::vector<double> med(mb);
  EXPECT(mr_prep_medians(p, med.data()) == 0, "medians");
  for (int k : {3, 5}) {
    std::vector<unsigned char> keep(n);
    int rounds = 0, nus = 0, nms = 0;
    long long kept = 0;
    EXPECT(mr_prep_shrink(p, k, k == 3, keep.data(), &rounds, &kept, &nus, &nms) == 0, "shrink");
    const long long cb[3] = {0, kept / 2, kept};
    std::vector<long long> fu(2 * (size_t)ub), fm(2 * (size_t)mb);
    EXPECT(mr_prep_first_appearance(p, 2, cb, fu.data(), fm.data()) == 0, "first_appearance");
    std::vector<int> umap(ub, 0), mmap(mb, 0);
    for (int a = 0; a < ub; ++a) umap[a] = a;
    for (int a = 0; a < mb; ++a) mmap[a] = a;
    std::vector<int> ou(kept), om(kept);
    std::vector<double> orr(kept);
    EXPECT(mr_prep_convert(p, umap.data(), mmap.data(), med.data(), ou.data(), om.data(),
                           orr.data()) == 0,
           "convert");
  }
  (void)mr_prep_last_ms(p);
  mr_prep_destroy(p);
}

static void run_similar() {
  const int nm = 120, nus = 500;
  std::mt19937 g(7);
  std::vector<long long> off(1, 0);
  std::vector<int> user;
  std::vector<unsigned char> r2;
  std::vector<unsigned long long> gm(nm);
  std::vector<unsigned char> hg(nm, 1);
  for (int mv = 0; mv < nm; ++mv) {
    for (int a = 0; a < nus; ++a)
      if ((g() % 100) < 20) {
        user.push_back(a);
        r2.push_back((unsigned char)(1 + g() % 10));
      }
    off.push_back((long long)user.size());
    gm[mv] = 1ull << (mv % 4);
  }
  hg[5] = 0;
  mr_similar* s = mr_similar_create(0, nm, nus, off.data(), user.data(), r2.data(), gm.data(),
                                    hg.data());
  EXPECT(s, "mr_similar_create");
  if (!s) return;
  std::vector<double> boost(200);
  for (int n = 0; n < 200; ++n) boost[n] = 1.0 + 0.001 * n;
  const int nr = 20;
  std::vector<int> oi(nm * nr), oc(nm);
  std::vector<double> os(nm * nr);
  EXPECT(mr_similar_find(s, nm, nullptr, boost.data(), (int)boost.size(), nr, oi.data(), os.data(),
                         oc.data()) == 0,
         "similar_find");
  (void)mr_similar_last_ms(s);
  mr_similar_destroy(s);
}

int main() {
  if (mr_device_count() < 1) {
    fprintf(stderr, "no GPU\n");
    return 2;
  }
  run_reference_abi();
  for (int k : {10, 33, 64, 128}) run_engine(k, k == 33 ? 64 : 2048);
  run_serving();
  run_prep();
  run_similar();
  printf("asan driver: %d failure(s)\n", g_fail);
  return g_fail ? 1 : 0;
}
