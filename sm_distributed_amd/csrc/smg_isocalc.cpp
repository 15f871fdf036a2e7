// Theoretical isotope patterns (host code of libsmg.so).
//
// Replaces the centroid generation behind sm/engine/isocalc_wrapper.py:37-70 (complete_isodist(parseSumFormula(
// sf + adduct), sigma, charge, pts_per_mz, centroid_kwargs={'weighted_bins': 5}) -> first six centroids) and the
// Spark fan-out of theor_peaks_gen.py:113-134 (a thread pool over (sf, adduct) strings).  The arithmetic of the
// third-party calculator is restated in oracle/isocalc_oracle.py (the contract, parity unpinned); this file
// follows it step for step so the two agree to floating-point rounding:
//   parse -> per-element binary powering of the isotope distribution -> product over elements in symbol order
//   (prune < PRUNE * max, merge runs closer than MERGE_TOL) -> cutoff 0.1 % -> charge -> truncated Gaussians on
//   the grid j / pts_per_mz (FWHM = sigma / 2.35482) -> local maxima, weighted centroids over +-weighted_bins.
// The profile is evaluated only on the grid segments the truncated Gaussians touch (padded by weighted_bins + 1
// zero points), which equals the dense grid of the oracle: everything outside is exactly zero.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/smg.h"

namespace smg {
void set_error(const char* fmt, ...);
}

namespace {

constexpr double ELECTRON_MASS = 0.00054857990946;
constexpr double FWHM_PER_SIGMA = 2.3548200450309493;
constexpr double PRUNE = 1e-9;
constexpr double MERGE_TOL = 1e-6;
constexpr double TRUNC_S = 6.0;
constexpr double CUTOFF_PERC = 0.1;

struct Iso {
  double m, p;
};
struct Element {
  const char* sym;
  std::vector<Iso> iso;  // ascending mass
};

// IUPAC/NIST masses and representative abundances (same table as oracle/isocalc_oracle.py ISOTOPES)
const std::vector<Element>& table() {
  static const std::vector<Element> t = {
      {"H", {{1.00782503207, 0.999885}, {2.0141017778, 0.000115}}},
      {"He", {{3.0160293191, 1.34e-06}, {4.00260325415, 0.99999866}}},
      {"Li", {{6.015122795, 0.0759}, {7.01600455, 0.9241}}},
      {"B", {{10.0129370, 0.199}, {11.0093054, 0.801}}},
      {"C", {{12.0, 0.9893}, {13.0033548378, 0.0107}}},
      {"N", {{14.0030740048, 0.99636}, {15.0001088982, 0.00364}}},
      {"O", {{15.99491461956, 0.99757}, {16.99913170, 0.00038}, {17.9991610, 0.00205}}},
      {"F", {{18.99840322, 1.0}}},
      {"Na", {{22.9897692809, 1.0}}},
      {"Mg", {{23.985041700, 0.7899}, {24.98583692, 0.1000}, {25.982592929, 0.1101}}},
      {"Al", {{26.98153863, 1.0}}},
      {"Si", {{27.9769265325, 0.92223}, {28.976494700, 0.04685}, {29.97377017, 0.03092}}},
      {"P", {{30.97376163, 1.0}}},
      {"S", {{31.97207100, 0.9499}, {32.97145876, 0.0075}, {33.96786690, 0.0425}, {35.96708076, 0.0001}}},
      {"Cl", {{34.96885268, 0.7576}, {36.96590259, 0.2424}}},
      {"K", {{38.96370668, 0.932581}, {39.96399848, 0.000117}, {40.96182576, 0.067302}}},
      {"Ca", {{39.96259098, 0.96941}, {41.95861801, 0.00647}, {42.9587666, 0.00135}, {43.9554818, 0.02086},
              {45.9536926, 4e-05}, {47.952534, 0.00187}}},
      {"Mn", {{54.9380451, 1.0}}},
      {"Fe", {{53.9396105, 0.05845}, {55.9349375, 0.91754}, {56.9353940, 0.02119}, {57.9332756, 0.00282}}},
      {"Co", {{58.9331950, 1.0}}},
      {"Ni", {{57.9353429, 0.680769}, {59.9307864, 0.262231}, {60.9310560, 0.011399}, {61.9283451, 0.036345},
              {63.9279660, 0.009256}}},
      {"Cu", {{62.9295975, 0.6915}, {64.9277895, 0.3085}}},
      {"Zn", {{63.9291422, 0.48268}, {65.9260334, 0.27975}, {66.9271273, 0.04102}, {67.9248442, 0.19024},
              {69.9253193, 0.00631}}},
      {"As", {{74.9215965, 1.0}}},
      {"Se", {{73.9224764, 0.0089}, {75.9192136, 0.0937}, {76.9199140, 0.0763}, {77.9173091, 0.2377},
              {79.9165213, 0.4961}, {81.9166994, 0.0873}}},
      {"Br", {{78.9183371, 0.5069}, {80.9162906, 0.4931}}},
      {"I", {{126.904473, 1.0}}},
      {"Au", {{196.9665687, 1.0}}},
      // the remaining decoy-adduct elements of fdr.py:8 (NIST isotope masses, IUPAC representative abundances)
      {"Be", {{9.0121822, 1.0}}},
      {"Ne", {{19.9924401754, 0.9048}, {20.99384668, 0.0027}, {21.991385114, 0.0925}}},
      {"Ar", {{35.967545106, 0.003365}, {37.9627324, 0.000632}, {39.9623831225, 0.996003}}},
      {"Sc", {{44.9559119, 1.0}}},
      {"Ti", {{45.9526316, 0.0825}, {46.9517631, 0.0744}, {47.9479463, 0.7372}, {48.94787, 0.0541}, {49.9447912, 0.0518}}},
      {"V", {{49.9471585, 0.0025}, {50.9439595, 0.9975}}},
      {"Cr", {{49.9460442, 0.04345}, {51.9405075, 0.83789}, {52.9406494, 0.09501}, {53.9388804, 0.02365}}},
      {"Ga", {{68.9255736, 0.60108}, {70.9247013, 0.39892}}},
      {"Ge", {{69.9242474, 0.2038}, {71.9220758, 0.2731}, {72.9234589, 0.0776}, {73.9211778, 0.3672}, {75.9214026, 0.0783}}},
      {"Kr", {{77.9203648, 0.00355}, {79.916379, 0.02286}, {81.9134836, 0.11593}, {82.914136, 0.115}, {83.911507, 0.56987}, {85.91061073, 0.17279}}},
      {"Rb", {{84.911789738, 0.7217}, {86.909180527, 0.2783}}},
      {"Sr", {{83.913425, 0.0056}, {85.9092602, 0.0986}, {86.9088771, 0.07}, {87.9056121, 0.8258}}},
      {"Y", {{88.9058483, 1.0}}},
      {"Zr", {{89.9047044, 0.5145}, {90.9056458, 0.1122}, {91.9050408, 0.1715}, {93.9063152, 0.1738}, {95.9082734, 0.028}}},
      {"Nb", {{92.9063781, 1.0}}},
      {"Mo", {{91.906811, 0.1477}, {93.9050883, 0.0923}, {94.9058421, 0.159}, {95.9046795, 0.1668}, {96.9060215, 0.0956}, {97.9054082, 0.2419}, {99.907477, 0.0967}}},
      {"Ru", {{95.907598, 0.0554}, {97.905287, 0.0187}, {98.9059393, 0.1276}, {99.9042195, 0.126}, {100.9055821, 0.1706}, {101.9043493, 0.3155}, {103.905433, 0.1862}}},
      {"Rh", {{102.905504, 1.0}}},
      {"Pd", {{101.905609, 0.0102}, {103.904036, 0.1114}, {104.905085, 0.2233}, {105.903486, 0.2733}, {107.903892, 0.2646}, {109.905153, 0.1172}}},
      {"Ag", {{106.905097, 0.51839}, {108.904752, 0.48161}}},
      {"Cd", {{105.906459, 0.0125}, {107.904184, 0.0089}, {109.9030021, 0.1249}, {110.9041781, 0.128}, {111.9027578, 0.2413}, {112.9044017, 0.1222}, {113.9033585, 0.2873}, {115.904756, 0.0749}}},
      {"In", {{112.904058, 0.0429}, {114.903878, 0.9571}}},
      {"Sn", {{111.904818, 0.0097}, {113.902779, 0.0066}, {114.903342, 0.0034}, {115.901741, 0.1454}, {116.902952, 0.0768}, {117.901603, 0.2422}, {118.903308, 0.0859}, {119.9021947, 0.3258}, {121.903439, 0.0463}, {123.9052739, 0.0579}}},
      {"Sb", {{120.9038157, 0.5721}, {122.904214, 0.4279}}},
      {"Te", {{119.90402, 0.0009}, {121.9030439, 0.0255}, {122.90427, 0.0089}, {123.9028179, 0.0474}, {124.9044307, 0.0707}, {125.9033117, 0.1884}, {127.9044631, 0.3174}, {129.9062244, 0.3408}}},
      {"Xe", {{123.905893, 0.000952}, {125.904274, 0.00089}, {127.9035313, 0.019102}, {128.9047794, 0.264006}, {129.903508, 0.04071}, {130.9050824, 0.212324}, {131.9041535, 0.269086}, {133.9053945, 0.104357}, {135.907219, 0.088573}}},
      {"Cs", {{132.905451933, 1.0}}},
      {"Ba", {{129.9063208, 0.00106}, {131.9050613, 0.00101}, {133.9045084, 0.02417}, {134.9056886, 0.06592}, {135.9045759, 0.07854}, {136.9058274, 0.11232}, {137.9052472, 0.71698}}},
      {"La", {{137.907112, 0.0009}, {138.9063533, 0.9991}}},
      {"Ce", {{135.907172, 0.00185}, {137.905991, 0.00251}, {139.9054387, 0.8845}, {141.909244, 0.11114}}},
      {"Pr", {{140.9076528, 1.0}}},
      {"Nd", {{141.9077233, 0.272}, {142.9098143, 0.122}, {143.9100873, 0.238}, {144.9125736, 0.083}, {145.9131169, 0.172}, {147.916893, 0.057}, {149.920891, 0.056}}},
      {"Sm", {{143.911999, 0.0307}, {146.9148979, 0.1499}, {147.9148227, 0.1124}, {148.9171847, 0.1382}, {149.9172755, 0.0738}, {151.9197324, 0.2675}, {153.9222093, 0.2275}}},
      {"Eu", {{150.9198502, 0.4781}, {152.9212303, 0.5219}}},
      {"Gd", {{151.919791, 0.002}, {153.9208656, 0.0218}, {154.922622, 0.148}, {155.9221227, 0.2047}, {156.9239601, 0.1565}, {157.9241039, 0.2484}, {159.9270541, 0.2186}}},
      {"Tb", {{158.9253468, 1.0}}},
      {"Dy", {{155.924283, 0.00056}, {157.924409, 0.00095}, {159.9251975, 0.02329}, {160.9269334, 0.18889}, {161.9267984, 0.25475}, {162.9287312, 0.24896}, {163.9291748, 0.2826}}},
      {"Ho", {{164.9303221, 1.0}}},
      {"Er", {{161.928778, 0.00139}, {163.9292, 0.01601}, {165.9302931, 0.33503}, {166.9320482, 0.22869}, {167.9323702, 0.26978}, {169.935464, 0.1491}}},
      {"Tm", {{168.9342133, 1.0}}},
      {"Yb", {{167.933897, 0.0013}, {169.9347618, 0.0304}, {170.9363258, 0.1428}, {171.9363815, 0.2183}, {172.9382108, 0.1613}, {173.9388621, 0.3183}, {175.9425717, 0.1276}}},
      {"Lu", {{174.9407718, 0.9741}, {175.9426863, 0.0259}}},
      {"Hf", {{173.940046, 0.0016}, {175.9414086, 0.0526}, {176.9432207, 0.186}, {177.9436988, 0.2728}, {178.9458161, 0.1362}, {179.94655, 0.3508}}},
      {"Ta", {{179.9474648, 0.00012}, {180.9479958, 0.99988}}},
      {"W", {{179.946704, 0.0012}, {181.9482042, 0.265}, {182.950223, 0.1431}, {183.9509312, 0.3064}, {185.9543641, 0.2843}}},
      {"Re", {{184.952955, 0.374}, {186.9557531, 0.626}}},
      {"Os", {{183.9524891, 0.0002}, {185.9538382, 0.0159}, {186.9557505, 0.0196}, {187.9558382, 0.1324}, {188.9581475, 0.1615}, {189.958447, 0.2626}, {191.9614807, 0.4078}}},
      {"Ir", {{190.960594, 0.373}, {192.9629264, 0.627}}},
      {"Pt", {{189.959932, 0.00014}, {191.961038, 0.00782}, {193.9626803, 0.32967}, {194.9647911, 0.33832}, {195.9649515, 0.25242}, {197.967893, 0.07163}}},
      {"Hg", {{195.965833, 0.0015}, {197.966769, 0.0997}, {198.9682799, 0.1687}, {199.968326, 0.231}, {200.9703023, 0.1318}, {201.970643, 0.2986}, {203.9734939, 0.0687}}},
      {"Tl", {{202.9723442, 0.2952}, {204.9744275, 0.7048}}},
      {"Pb", {{203.9730436, 0.014}, {205.9744653, 0.241}, {206.9758969, 0.221}, {207.9766521, 0.524}}},
      {"Bi", {{208.9803987, 1.0}}},
      {"Th", {{232.0380553, 1.0}}},
      {"U", {{234.0409521, 5.4e-05}, {235.0439299, 0.007204}, {238.0507882, 0.992742}}},
  };
  return t;
}

const Element* find_element(const std::string& s) {
  for (const auto& e : table())
    if (s == e.sym) return &e;
  return nullptr;
}

// ---- parser (oracle parse_sum_formula): tokens = element | ( | ) | digits | + | -
struct Parser {
  const char* s;
  size_t n, pos = 0;
  std::string err;
  enum Kind { ELEM, LP, RP, NUM, SIGN, END, BAD };
  Kind peek(std::string* text = nullptr) const {
    if (pos >= n) return END;
    const char c = s[pos];
    if (c >= 'A' && c <= 'Z') {
      size_t e = pos + 1;
      while (e < n && s[e] >= 'a' && s[e] <= 'z') ++e;
      if (text) text->assign(s + pos, e - pos);
      return ELEM;
    }
    if (c == '(') return LP;
    if (c == ')') return RP;
    if (c >= '0' && c <= '9') return NUM;
    if (c == '+' || c == '-') return SIGN;
    return BAD;
  }
  long long number() {
    long long v = 0;
    while (pos < n && s[pos] >= '0' && s[pos] <= '9') {
      v = v * 10 + (s[pos] - '0');
      if (v > (1ll << 40)) v = 1ll << 40;  // absurd counts are rejected by the caller
      ++pos;
    }
    return v;
  }
  bool group(std::map<std::string, long long>& out) {
    int items = 0;
    while (true) {
      std::string tok;
      const Kind k = peek(&tok);
      if (k == END || k == RP || k == SIGN) break;
      std::map<std::string, long long> sub;
      if (k == LP) {
        ++pos;
        if (!group(sub)) return false;
        if (peek() != RP) {
          err = "unbalanced parenthesis";
          return false;
        }
        ++pos;
      } else if (k == ELEM) {
        if (!find_element(tok)) {
          err = "unknown element '" + tok + "'";
          return false;
        }
        sub[tok] = 1;
        pos += tok.size();
      } else if (k == NUM) {
        err = "misplaced count";
        return false;
      } else {
        err = "unexpected character";
        return false;
      }
      long long mult = 1;
      if (peek() == NUM) mult = number();
      for (const auto& kv : sub) out[kv.first] += kv.second * mult;
      ++items;
    }
    if (items == 0) {
      err = "empty group";
      return false;
    }
    return true;
  }
  bool formula(std::map<std::string, long long>& total) {
    if (n == 0) {
      err = "empty formula";
      return false;
    }
    int sign = 1;
    if (peek() == SIGN) {
      sign = s[pos] == '-' ? -1 : 1;
      ++pos;
    }
    while (true) {
      std::map<std::string, long long> g;
      if (!group(g)) return false;
      for (const auto& kv : g) total[kv.first] += sign * kv.second;
      const Kind k = peek();
      if (k == END) break;
      if (k != SIGN) {
        err = k == BAD ? "unexpected character" : "unbalanced parenthesis";
        return false;
      }
      sign = s[pos] == '-' ? -1 : 1;
      ++pos;
      if (peek() == END) {
        err = "dangling sign";
        return false;
      }
    }
    for (auto it = total.begin(); it != total.end();) {
      if (it->second < 0) {
        err = "negative element count";
        return false;
      }
      if (it->second > (1 << 20)) {
        err = "element count too large";
        return false;
      }
      it = it->second == 0 ? total.erase(it) : std::next(it);
    }
    if (total.empty()) {
      err = "no atoms";
      return false;
    }
    return true;
  }
};

// product of two distributions (oracle _convolve): pairs in (i, j) order, prune, stable sort, merge runs
std::vector<Iso> convolve(const std::vector<Iso>& a, const std::vector<Iso>& b) {
  std::vector<Iso> c;
  c.reserve(a.size() * b.size());
  double pmax = 0.0;
  for (const auto& x : a)
    for (const auto& y : b) {
      c.push_back({x.m + y.m, x.p * y.p});
      pmax = std::max(pmax, x.p * y.p);
    }
  const double thr = PRUNE * pmax;
  c.erase(std::remove_if(c.begin(), c.end(), [&](const Iso& v) { return !(v.p >= thr); }), c.end());
  std::stable_sort(c.begin(), c.end(), [](const Iso& x, const Iso& y) { return x.m < y.m; });
  std::vector<Iso> out;
  size_t i = 0;
  while (i < c.size()) {
    size_t j = i + 1;
    while (j < c.size() && !(c[j].m - c[j - 1].m > MERGE_TOL)) ++j;
    double ps = 0.0, mps = 0.0;
    for (size_t k = i; k < j; ++k) {
      ps += c[k].p;
      mps += c[k].m * c[k].p;
    }
    out.push_back({mps / ps, ps});
    i = j;
  }
  return out;
}

std::vector<Iso> element_power(const Element& e, long long n) {
  std::vector<Iso> r = {{0.0, 1.0}}, base = e.iso;
  while (n) {
    if (n & 1) r = convolve(r, base);
    n >>= 1;
    if (n) base = convolve(base, base);
  }
  return r;
}

struct Centroid {
  double mz, in;
};

// all centroids of one formula string; false + err on an invalid formula
bool centroids(const char* sf, int charge, double sigma, int pts, int wb, std::vector<Centroid>& out,
               std::string& err) {
  out.clear();
  Parser ps{sf, strlen(sf)};
  std::map<std::string, long long> counts;
  if (!ps.formula(counts)) {
    err = ps.err;
    return false;
  }
  std::vector<Iso> d = {{0.0, 1.0}};
  for (const auto& kv : counts) d = convolve(d, element_power(*find_element(kv.first), kv.second));
  double pmax = 0.0;
  for (const auto& v : d) pmax = std::max(pmax, v.p);
  const double cut = CUTOFF_PERC / 100.0 * pmax;
  std::vector<Iso> pk;
  for (const auto& v : d)
    if (v.p >= cut) pk.push_back(v);
  if (charge != 0)
    for (auto& v : pk) v.m = (v.m - charge * ELECTRON_MASS) / std::abs(charge);
  const double s = sigma / FWHM_PER_SIGMA / FWHM_PER_SIGMA;
  const double inv2s2 = 1.0 / (2.0 * s * s);
  (void)inv2s2;
  const double pts_d = (double)pts;
  const size_t np_ = pk.size();
  std::vector<long long> lo(np_), hi(np_);
  for (size_t i = 0; i < np_; ++i) {
    lo[i] = (long long)std::ceil((pk[i].m - TRUNC_S * s) * pts_d);
    hi[i] = (long long)std::floor((pk[i].m + TRUNC_S * s) * pts_d);
  }
  // segments of the padded supports (peaks ascend in mass, so supports start in ascending order)
  std::vector<double> y;
  size_t i = 0;
  while (i < np_) {
    long long a = lo[i] - wb - 1, b = hi[i] + wb + 1;
    size_t j = i + 1;
    while (j < np_ && lo[j] - wb - 1 <= b) {
      b = std::max(b, hi[j] + wb + 1);
      ++j;
    }
    y.assign((size_t)(b - a + 1), 0.0);
    for (size_t k = i; k < j; ++k) {
      for (long long g = lo[k]; g <= hi[k]; ++g) {
        const double x = (double)g / pts_d;
        const double dd = x - pk[k].m;
        y[(size_t)(g - a)] += pk[k].p * std::exp(-(dd * dd) / (2.0 * s * s));
      }
    }
    const long long len = b - a + 1;
    for (long long q = 1; q + 1 < len; ++q) {
      const double v = y[(size_t)q];
      if (v > 0.0 && y[(size_t)q - 1] < v && v >= y[(size_t)q + 1]) {
        double sxy = 0.0, sy = 0.0;
        for (long long r = q - wb; r <= q + wb; ++r) {
          const double x = (double)(a + r) / pts_d;
          sxy += x * y[(size_t)r];
          sy += y[(size_t)r];
        }
        out.push_back({sxy / sy, v});
      }
    }
    i = j;
  }
  double imax = 0.0;
  for (const auto& c : out) imax = std::max(imax, c.in);
  for (auto& c : out) c.in = c.in * (100.0 / imax);
  return true;
}

bool check_params(double sigma, int pts, int wb) {
  return std::isfinite(sigma) && sigma > 0.0 && pts > 0 && wb >= 0 && wb <= 1000 &&
         sigma / FWHM_PER_SIGMA / FWHM_PER_SIGMA * TRUNC_S * pts < 1e7;
}

}  // namespace

extern "C" {

int smg_isotope_centroids(const char* sf_adduct, int32_t charge, double sigma, int32_t pts_per_mz,
                          int32_t weighted_bins, int32_t cap, double* mzs, double* ints, int32_t* n_out) {
  if (!sf_adduct || !n_out || cap < 0 || (cap > 0 && (!mzs || !ints)) ||
      !check_params(sigma, pts_per_mz, weighted_bins)) {
    smg::set_error("smg_isotope_centroids: bad arguments");
    return SMG_ERR_INVALID;
  }
  std::vector<Centroid> c;
  std::string err;
  *n_out = 0;
  if (!centroids(sf_adduct, charge, sigma, pts_per_mz, weighted_bins, c, err)) {
    smg::set_error("invalid sum formula '%s': %s", sf_adduct, err.c_str());
    return SMG_ERR_INVALID;
  }
  const int n = (int)std::min<size_t>(c.size(), (size_t)cap);
  for (int k = 0; k < n; ++k) {
    mzs[k] = c[(size_t)k].mz;
    ints[k] = c[(size_t)k].in;
  }
  *n_out = n;
  return SMG_OK;
}

int smg_isotope_centroids_batch(const char* formulas, const int64_t* offsets, int64_t n, int32_t charge,
                                double sigma, int32_t pts_per_mz, int32_t weighted_bins, int32_t cap,
                                double* mzs, double* ints, int32_t* n_out, int32_t n_threads) {
  if (n < 0 || cap < 0 || (n > 0 && (!formulas || !offsets || !n_out || (cap > 0 && (!mzs || !ints)))) ||
      !check_params(sigma, pts_per_mz, weighted_bins)) {
    smg::set_error("smg_isotope_centroids_batch: bad arguments");
    return SMG_ERR_INVALID;
  }
  if (n == 0) return SMG_OK;
  int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
  nt = (int)std::min<int64_t>(nt, n);
  std::atomic<int64_t> next{0};
  auto work = [&]() {
    std::vector<Centroid> c;
    std::string err, sf;
    while (true) {
      const int64_t i = next.fetch_add(1);
      if (i >= n) break;
      sf.assign(formulas + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
      if (!centroids(sf.c_str(), charge, sigma, pts_per_mz, weighted_bins, c, err)) {
        n_out[i] = -1;
        continue;
      }
      const int m = (int)std::min<size_t>(c.size(), (size_t)cap);
      for (int k = 0; k < m; ++k) {
        mzs[i * cap + k] = c[(size_t)k].mz;
        ints[i * cap + k] = c[(size_t)k].in;
      }
      n_out[i] = m;
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  return SMG_OK;
}

}  // extern "C"
