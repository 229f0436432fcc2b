// Host-side reader for GENPARMMP.TBL / SOILPARMMP.TBL / VEGPARMMP.TBL.
//
// Same block/tag rules and list-directed field semantics as the reference
// readers:
//   block finder  core/module_noahmp_utils.f90:200-237  ("&NAME" / "&NAME#TAG",
//                 first list-directed item of each record, blank records skipped)
//   table reader  core/module_noahmp_utils.f90:56-97    (row count = first item of
//                 the next record, then that many raw records; rows are assigned
//                 in order, the leading index column is ignored)
//   scalar/vector core/module_noahmp_utils.f90:100-197
//   gen / soil / veg tables and derived KDT, FRZX
//                 core/module_noahmp_gen_param.f90:51-89
//                 core/module_noahmp_soil_param.f90:31-72  (FRZX keeps the
//                 reference's integer 0468 divisor, SURVEY hazard H1)
//                 core/module_noahmp_veg_param.f90:77-161
// Unread entries keep the reference initial values (nan4 / -1 / 0).
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "noahmp_engine.h"

namespace {

float nan4() {  // transfer(-4194304_i4, 1.0_r4), core/module_noahmp_const.f90:13
  int32_t bits = -4194304;
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

struct Tbl {
  std::vector<std::string> rec;
  bool load(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::string line;
    while (std::getline(f, line)) {
      while (!line.empty() && (line.back() == '\r' || line.back() == '\n')) line.pop_back();
      rec.push_back(line);
    }
    return true;
  }
};

// list-directed items of one record: separators blank/comma/tab, '/' ends
// the record, quoted strings are one item
std::vector<std::string> items(const std::string& s) {
  std::vector<std::string> out;
  size_t i = 0, n = s.size();
  while (i < n) {
    char ch = s[i];
    if (ch == ' ' || ch == '\t' || ch == ',') {
      ++i;
      continue;
    }
    if (ch == '/') break;
    if (ch == '\'' || ch == '"') {
      size_t j = s.find(ch, i + 1);
      if (j == std::string::npos) j = n;
      out.push_back(s.substr(i + 1, j - i - 1));
      i = j + 1;
      continue;
    }
    size_t j = i;
    while (j < n && s[j] != ' ' && s[j] != '\t' && s[j] != ',' && s[j] != '/') ++j;
    out.push_back(s.substr(i, j - i));
    i = j;
  }
  return out;
}

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t");
  if (a == std::string::npos) return "";
  size_t b = s.find_last_not_of(" \t");
  return s.substr(a, b - a + 1);
}

// noahmp_ptable_find_name_tag: index of the header record, or -1
long find_block(const Tbl& t, const std::string& name, const std::string& tag) {
  const std::string nm = trim(name), tg = trim(tag);
  if (nm.empty()) return -1;
  for (size_t r = 0; r < t.rec.size(); ++r) {
    std::vector<std::string> it = items(t.rec[r]);
    if (it.empty()) continue;  // blank record: list-directed read moves on
    const std::string& sb = it[0];
    if (sb.empty() || sb[0] != '&') continue;
    size_t loc = sb.find('#');
    if (loc == std::string::npos && tg.empty()) {
      if (trim(sb.substr(1)) == nm) return (long)r;
    } else if (loc != std::string::npos && !tg.empty()) {
      if (trim(sb.substr(1, loc - 1)) == nm && trim(sb.substr(loc + 1)) == tg) return (long)r;
    }
  }
  return -1;
}

// list-directed read of n items starting at record r (spanning records);
// returns the index of the record after the last one consumed, or -1
long read_items(const Tbl& t, long r, size_t n, std::vector<std::string>& out) {
  out.clear();
  while (out.size() < n) {
    if (r >= (long)t.rec.size()) return -1;
    std::vector<std::string> it = items(t.rec[r]);
    for (auto& s : it) {
      if (out.size() < n) out.push_back(s);
    }
    ++r;
  }
  return r;
}

bool to_real(const std::string& s, float& v) {
  if (s.empty()) return false;
  std::string t = s;
  for (auto& ch : t)
    if (ch == 'd' || ch == 'D') ch = 'e';
  char* end = nullptr;
  v = std::strtof(t.c_str(), &end);
  return end && *end == '\0';
}
bool to_int(const std::string& s, int32_t& v) {
  if (s.empty()) return false;
  char* end = nullptr;
  long x = std::strtol(s.c_str(), &end, 10);
  if (!end || *end != '\0') return false;
  v = (int32_t)x;
  return true;
}

// scalar / vector reads (noahmp_ptable_read_real0d/1d, int0d)
bool read_reals(const Tbl& t, const char* name, const char* tag, float* v, size_t n) {
  long r = find_block(t, name, tag);
  if (r < 0) return false;
  std::vector<std::string> it;
  if (read_items(t, r + 1, n, it) < 0) return false;
  for (size_t i = 0; i < n; ++i)
    if (!to_real(it[i], v[i])) return false;
  return true;
}
bool read_int(const Tbl& t, const char* name, const char* tag, int32_t& v) {
  long r = find_block(t, name, tag);
  if (r < 0) return false;
  std::vector<std::string> it;
  if (read_items(t, r + 1, 1, it) < 0) return false;
  return to_int(it[0], v);
}

// noahmp_ptable_read_tablestr: the raw row records of a table
bool read_table(const Tbl& t, const char* name, const char* tag, size_t maxrow,
                std::vector<std::string>& rows, int32_t& nrow) {
  long r = find_block(t, name, tag);
  if (r < 0) return false;
  std::vector<std::string> it;
  long next = read_items(t, r + 1, 1, it);
  if (next < 0 || !to_int(it[0], nrow)) return false;
  if (nrow < 0 || (size_t)nrow > maxrow) return false;
  rows.clear();
  for (int32_t i = 0; i < nrow; ++i) {
    if (next + i >= (long)t.rec.size()) return false;
    rows.push_back(t.rec[next + i]);
  }
  return true;
}

// one table row: leading index, then a sequence of (int|real) fields
struct Field {
  bool is_int;
  void* dst;
};
bool parse_row(const std::string& row, const std::vector<Field>& f) {
  std::vector<std::string> it = items(row);
  if (it.size() < f.size() + 1) return false;
  int32_t idx;
  if (!to_int(it[0], idx)) return false;
  for (size_t i = 0; i < f.size(); ++i) {
    if (f[i].is_int) {
      if (!to_int(it[i + 1], *(int32_t*)f[i].dst)) return false;
    } else {
      if (!to_real(it[i + 1], *(float*)f[i].dst)) return false;
    }
  }
  return true;
}

Field R(float& x) { return Field{false, &x}; }
Field I(int32_t& x) { return Field{true, &x}; }

}  // namespace

extern "C" int nmp_read_tables(const char* tbl_dir, const char* soil_tag, const char* veg_tag,
                               nmp_params* P) {
  if (!tbl_dir || !soil_tag || !veg_tag || !P) return NMP_E_ARG;
  // reference initial values
  {
    float* fp = reinterpret_cast<float*>(P);
    const size_t nf = offsetof(nmp_params, nslptyp) / sizeof(float);
    const float q = nan4();
    for (size_t i = 0; i < nf; ++i) fp[i] = q;
    P->nslptyp = P->nsltyp = P->nsoilcol = P->nlutyp = 0;
    P->isurban = P->iswater = P->isbarren = P->isice = P->isegblf = -1;
    for (int i = 0; i < NMP_MLUTYP; ++i) {
      P->nroot[i] = -1;
      P->c3c4[i] = 0;
    }
  }
  const std::string dir(tbl_dir);
  Tbl gen, soil, veg;
  if (!gen.load(dir + "/GENPARMMP.TBL") || !soil.load(dir + "/SOILPARMMP.TBL") ||
      !veg.load(dir + "/VEGPARMMP.TBL"))
    return NMP_E_TABLE;
  std::vector<std::string> rows;

  // ---- GENPARMMP.TBL: gen_param.f90:51-89
  if (!read_table(gen, "SLOPE", "", NMP_MSLOPETYP, rows, P->nslptyp)) return NMP_E_TABLE;
  for (int i = 0; i < P->nslptyp; ++i)
    if (!parse_row(rows[i], {R(P->slope[i])})) return NMP_E_TABLE;
  struct {
    const char* n;
    float* v;
    size_t k;
  } gs[] = {{"CSOIL", &P->csoil, 1},   {"DKREF", &P->dkref, 1},     {"KDTREF", &P->kdtref, 1},
            {"FRZK", &P->frzk, 1},     {"ZBOT", &P->zbot, 1},       {"CZIL", &P->czil, 1},
            {"TIMEAN", &P->timean, 1}, {"FSATMAX", &P->fsatmax, 1}, {"MLTFCT", &P->mltfct, 1},
            {"Z0SNO", &P->z0sno, 1},   {"SSI", &P->ssi, 1},         {"SWEMAX", &P->swemax, 1},
            {"ALBICE", P->albice, 2},  {"ALBLAKE", P->alblake, 2},  {"OMEGAS", P->omegas, 2},
            {"BETADS", &P->betads, 1}, {"BETAIS", &P->betais, 1},   {"EMSSOIL", &P->emssoil, 1},
            {"EMSLAKE", &P->emslake, 1}};
  for (auto& g : gs)
    if (!read_reals(gen, g.n, "", g.v, g.k)) return NMP_E_TABLE;

  // ---- SOILPARMMP.TBL: soil_param.f90:31-72
  if (!read_table(soil, "PARM", soil_tag, NMP_MSLTYP, rows, P->nsltyp)) return NMP_E_TABLE;
  for (int i = 0; i < P->nsltyp; ++i)
    if (!parse_row(rows[i], {R(P->bexp[i]), R(P->smcmax[i]), R(P->smcref[i]), R(P->smcwlt[i]),
                             R(P->psisat[i]), R(P->dksat[i]), R(P->dwsat[i]), R(P->quartz[i])}))
      return NMP_E_TABLE;
  for (int i = 0; i < NMP_MSLTYP; ++i) {
    P->kdt[i] = P->kdtref * P->dksat[i] / P->dkref;
    if (P->smcref[i] > 0.0f) P->frzx[i] = P->frzk * (P->smcmax[i] / P->smcref[i]) * (0.412f / 468.0f);
  }
  if (!read_table(soil, "COLOR", "", NMP_MSLCOL, rows, P->nsoilcol)) return NMP_E_TABLE;
  for (int i = 0; i < P->nsoilcol; ++i)
    if (!parse_row(rows[i], {R(P->albsat[i][0]), R(P->albsat[i][1]), R(P->albdry[i][0]),
                             R(P->albdry[i][1])}))
      return NMP_E_TABLE;

  // ---- VEGPARMMP.TBL: veg_param.f90:77-161
  if (!read_int(veg, "ISURBAN", veg_tag, P->isurban) ||
      !read_int(veg, "ISWATER", veg_tag, P->iswater) ||
      !read_int(veg, "ISBARREN", veg_tag, P->isbarren) ||
      !read_int(veg, "ISICE", veg_tag, P->isice) || !read_int(veg, "ISEGBLF", veg_tag, P->isegblf))
    return NMP_E_TABLE;
  int32_t n;
  if (!read_table(veg, "RAD", veg_tag, NMP_MLUTYP, rows, n)) return NMP_E_TABLE;
  P->nlutyp = n;
  for (int i = 0; i < n; ++i)
    if (!parse_row(rows[i], {R(P->xl[i]), R(P->rhol[i][0]), R(P->rhol[i][1]), R(P->rhos[i][0]),
                             R(P->rhos[i][1]), R(P->taul[i][0]), R(P->taul[i][1]),
                             R(P->taus[i][0]), R(P->taus[i][1])}))
      return NMP_E_TABLE;
  if (!read_table(veg, "LAI12M", veg_tag, NMP_MLUTYP, rows, n)) return NMP_E_TABLE;
  P->nlutyp = n;
  for (int i = 0; i < n; ++i) {
    std::vector<Field> f;
    for (int m = 0; m < 12; ++m) f.push_back(R(P->lai12m[i][m]));
    if (!parse_row(rows[i], f)) return NMP_E_TABLE;
  }
  if (!read_table(veg, "SAI12M", veg_tag, NMP_MLUTYP, rows, n)) return NMP_E_TABLE;
  P->nlutyp = n;
  for (int i = 0; i < n; ++i) {
    std::vector<Field> f;
    for (int m = 0; m < 12; ++m) f.push_back(R(P->sai12m[i][m]));
    if (!parse_row(rows[i], f)) return NMP_E_TABLE;
  }
  if (!read_table(veg, "DVEG", veg_tag, NMP_MLUTYP, rows, n)) return NMP_E_TABLE;
  P->nlutyp = n;
  for (int i = 0; i < n; ++i)
    if (!parse_row(rows[i], {R(P->sla[i]), R(P->dilefc[i]), R(P->dilefw[i]), R(P->fragr[i]),
                             R(P->ltovrc[i]), R(P->wrrat[i]), R(P->wdpool[i]), R(P->tdlef[i])}))
      return NMP_E_TABLE;
  if (!read_table(veg, "PHYS", veg_tag, NMP_MLUTYP, rows, n)) return NMP_E_TABLE;
  P->nlutyp = n;
  for (int i = 0; i < n; ++i)
    if (!parse_row(rows[i], {I(P->nroot[i]), R(P->canwmxp[i]), R(P->dleaf[i]), R(P->z0mvt[i]),
                             R(P->hvt[i]), R(P->hvb[i]), R(P->den[i]), R(P->rcrown[i]),
                             R(P->cwpvt[i])}))
      return NMP_E_TABLE;
  if (!read_table(veg, "PHOTO", veg_tag, NMP_MLUTYP, rows, n)) return NMP_E_TABLE;
  P->nlutyp = n;
  for (int i = 0; i < n; ++i)
    if (!parse_row(rows[i],
                   {I(P->c3c4[i]), R(P->rgl[i]), R(P->hs[i]), R(P->kc25[i]), R(P->akc[i]),
                    R(P->ko25[i]), R(P->ako[i]), R(P->vcmx25[i]), R(P->avcmx[i]), R(P->bp[i]),
                    R(P->rsmax[i]), R(P->rsmin[i]), R(P->mp[i]), R(P->qe25[i]), R(P->aqe[i]),
                    R(P->rmf25[i]), R(P->rms25[i]), R(P->rmr25[i]), R(P->folnmx[i]),
                    R(P->topt[i]), R(P->tmin[i]), R(P->arm[i]), R(P->mrp[i])}))
      return NMP_E_TABLE;
  if (!read_table(veg, "VOC", veg_tag, NMP_MLUTYP, rows, n)) return NMP_E_TABLE;
  P->nlutyp = n;
  for (int i = 0; i < n; ++i)
    if (!parse_row(rows[i], {R(P->slarea[i]), R(P->eps[i][0]), R(P->eps[i][1]), R(P->eps[i][2]),
                             R(P->eps[i][3]), R(P->eps[i][4])}))
      return NMP_E_TABLE;
  return NMP_OK;
}
