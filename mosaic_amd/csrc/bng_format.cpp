// BNG StringType cell ids (BNG's default cell-id type, BNGIndexSystem.scala:30).
//
// mgpu_bng_format replaces BNGIndexSystem.format (BNGIndexSystem.scala:119-134)
// with indexDigits = Long.toString (:440-442); mgpu_bng_parse replaces
// BNGIndexSystem.parse and re-encodes with the same Double arithmetic as encode
// (:540-553).  Host code: string formatting is an output-side conversion of the
// id column (IndexSystem.serializeCellId, IndexSystem.scala:61-70).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "error.h"
#include "../../include/mosaic_gpu.h"
#include "bng_core.h"

namespace {

const char* kLetters[14][8] = {
    {"SV", "SW", "SX", "SY", "SZ", "TV", "TW", "TX"}, {"SQ", "SR", "SS", "ST", "SU", "TQ", "TR", "TS"},
    {"SL", "SM", "SN", "SO", "SP", "TL", "TM", "TN"}, {"SF", "SG", "SH", "SJ", "SK", "TF", "TG", "TH"},
    {"SA", "SB", "SC", "SD", "SE", "TA", "TB", "TC"}, {"NV", "NW", "NX", "NY", "NZ", "OV", "OW", "OX"},
    {"NQ", "NR", "NS", "NT", "NU", "OQ", "OR", "OS"}, {"NL", "NM", "NN", "NO", "NP", "OL", "OM", "ON"},
    {"NF", "NG", "NH", "NJ", "NK", "OF", "OG", "OH"}, {"NA", "NB", "NC", "ND", "NE", "OA", "OB", "OC"},
    {"HV", "HW", "HX", "HY", "HZ", "JV", "JW", "JX"}, {"HQ", "HR", "HS", "HT", "HU", "JQ", "JR", "JS"},
    {"HL", "HM", "HN", "HO", "HP", "JL", "JM", "JN"}, {"HF", "HG", "HH", "HJ", "HK", "JF", "JG", "JH"}};
const char* kQuadrants[5] = {"", "SW", "NW", "NE", "SE"};  // parse only

// the shared host/device formatter (bng_core.h)
int format_one(int64_t id, char* out) { return mgpu::bng::format_cell(id, out); }

double pow10d(int k) {
  double r = 1;
  for (int i = 0; i < k; i++) r *= 10;
  return r;
}

int64_t encode(int eL, int nL, int eB, int nB, int q, int nP, int res) {
  double idP = pow10d(5 + 2 * nP - 2), eLS = pow10d(3 + 2 * nP - 2), nLS = pow10d(1 + 2 * nP - 2);
  double eS = pow10d(nP), nS = 10;
  double id = res == -1 ? (idP + eL * eLS) / 100 + q : idP + eL * eLS + nL * nLS + eB * eS + nB * nS + q;
  return mgpu::bng::d2l(id);
}

bool parse_one(const char* s, int64_t len, int64_t* out) {
  if (len < 1) return false;
  char pre[3] = {s[0], len >= 2 ? s[1] : 'V', 0};
  int row = -1, col = -1;
  for (int r = 0; r < 14 && row < 0; r++)
    for (int c = 0; c < 8; c++)
      if (!strcmp(kLetters[r][c], pre)) {
        row = r;
        col = c;
        break;
      }
  if (row < 0) return false;  // letterMap.find(...).get throws
  if (len == 1) {
    *out = encode(col, 0, 0, 0, 0, 1, -1);
    return true;
  }
  int q = 0;
  if (len > 2) {
    for (int k = 1; k < 5; k++)
      if (s[len - 2] == kQuadrants[k][0] && s[len - 1] == kQuadrants[k][1]) q = k;
  }
  int64_t db = 2, de = q > 0 ? len - 2 : len;
  if (de <= db) {
    *out = encode(col, row, 0, 0, q, 1, -2);
    return true;
  }
  int64_t nd = de - db;
  int64_t half = nd / 2;
  long long eBin = 0, nBin = 0;
  for (int64_t i = db; i < de - half; i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    eBin = eBin * 10 + (s[i] - '0');
  }
  for (int64_t i = de - half; i < de; i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    nBin = nBin * 10 + (s[i] - '0');
  }
  if (half == 0) return false;  // "".toInt throws NumberFormatException
  int nP = (int)(nd / 2 + 1);
  int res = q == 0 ? nP + 1 : -nP;
  *out = encode(col, row, (int)eBin, (int)nBin, q, nP, res);
  return true;
}

}  // namespace

extern "C" {

int32_t mgpu_bng_format(const int64_t* cells, int64_t n, char* out, int64_t out_bytes, int64_t* out_offsets) {
  if (n < 0 || (n > 0 && (!cells || !out_offsets))) return mgpu::set_error(MGPU_E_INVALID_ARG, "bng_format: bad arguments");
  int64_t pos = 0;
  char buf[32];
  out_offsets[0] = 0;
  for (int64_t i = 0; i < n; i++) {
    int len = format_one(cells[i], buf);
    if (len < 0) return mgpu::set_error(MGPU_E_INVALID_ARG, "BNG cell id %lld has no string form", (long long)cells[i]);
    if (pos + len > out_bytes) return mgpu::set_error(MGPU_E_CAPACITY, "bng_format: output buffer too small");
    memcpy(out + pos, buf, len);
    pos += len;
    out_offsets[i + 1] = pos;
  }
  return MGPU_OK;
}

int32_t mgpu_bng_parse(const char* ids, const int64_t* offsets, int64_t n, int64_t* out_cells) {
  if (n < 0 || (n > 0 && (!ids || !offsets || !out_cells))) return mgpu::set_error(MGPU_E_INVALID_ARG, "bng_parse: bad arguments");
  for (int64_t i = 0; i < n; i++)
    if (!parse_one(ids + offsets[i], offsets[i + 1] - offsets[i], &out_cells[i]))
      return mgpu::set_error(MGPU_E_INVALID_ARG, "not a BNG cell id: %.*s", (int)(offsets[i + 1] - offsets[i]), ids + offsets[i]);
  return MGPU_OK;
}

}  // extern "C"
