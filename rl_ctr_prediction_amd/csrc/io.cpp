// Binary on-disk batch format: the reference's encoded CSV
// (`label,idx_1,...,idx_F` per line, written by src/encode/data_.py:85 and parsed with
// pandas at all_main/pretrain_main.py:50-53, or with islice + str.split per line at
// hybrid_td3_main_per_v10.py:348-351) converted once into a memory-mappable int32 matrix.
//
// File layout (little-endian):
//   [0, 64)   header: char magic[8] = "CTRBIN01"; int64 rows; int32 cols (= 1 + F);
//             int32 reserved (0); int64 max_id (largest feature id seen, -1 if none);
//             int64 data_offset (= 64); zero padding
//   [64, ..)  int32 [rows][cols] row-major: column 0 the label, columns 1..F the feature ids
// The same values the reference's `pd.read_csv(...).values.astype(int)` produces, so
// `libsvm_dataset(data[:, 1:], data[:, 0])` is unchanged; readers map the file (numpy
// memmap) and copy whole batches host -> device without parsing.
//
// The converter streams: the input is read in 16 MiB blocks and rows are written as they
// are parsed (constant memory for any file size); ragged rows, non-integer tokens and
// values outside int32 fail with the 1-based line number.
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "ctr_common.h"

namespace {

constexpr char kMagic[8] = {'C', 'T', 'R', 'B', 'I', 'N', '0', '1'};
constexpr int64_t kHeader = 64;

struct Header {
  char magic[8];
  int64_t rows;
  int32_t cols;
  int32_t reserved;
  int64_t max_id;
  int64_t data_offset;
  char pad[kHeader - 40];
};
static_assert(sizeof(Header) == kHeader, "64-byte header");

struct File {
  FILE* f = nullptr;
  ~File() {
    if (f) fclose(f);
  }
};

}  // namespace

extern "C" int ctr_csv_to_bin(const char* csv_path, const char* bin_path, int64_t* rows_out,
                              int32_t* cols_out, int64_t* max_id_out) {
  CTR_REQUIRE(csv_path && bin_path, "ctr_csv_to_bin: null path");
  File in, out;
  in.f = fopen(csv_path, "rb");
  CTR_REQUIRE(in.f, "ctr_csv_to_bin: cannot open %s: %s", csv_path, strerror(errno));
  out.f = fopen(bin_path, "wb");
  CTR_REQUIRE(out.f, "ctr_csv_to_bin: cannot create %s: %s", bin_path, strerror(errno));
  Header h;
  memset(&h, 0, sizeof(h));
  memcpy(h.magic, kMagic, 8);
  h.max_id = -1;
  h.data_offset = kHeader;
  CTR_REQUIRE(fwrite(&h, sizeof(h), 1, out.f) == 1, "ctr_csv_to_bin: write failed");

  std::vector<char> buf(16 << 20);
  std::vector<int32_t> row, wbuf;
  wbuf.reserve(1 << 20);
  int64_t line = 0, rows = 0;
  int32_t cols = -1;
  // token state, carried across block boundaries
  bool in_num = false, neg = false, any_digit = false, line_has_data = false;
  int64_t val = 0;
  auto end_token = [&]() -> bool {
    if (!in_num) return true;
    if (!any_digit) return false;
    const int64_t v = neg ? -val : val;
    if (v < INT32_MIN || v > INT32_MAX) return false;
    row.push_back((int32_t)v);
    if (row.size() > 1 && v > h.max_id) h.max_id = v;
    in_num = neg = any_digit = false;
    val = 0;
    return true;
  };
  auto end_line = [&]() -> int {
    ++line;
    if (!end_token()) {
      ::ctr::set_error("ctr_csv_to_bin: %s line %lld: bad integer", csv_path, (long long)line);
      return CTR_ERR_INVALID;
    }
    if (!line_has_data) {  // blank line (e.g. a trailing newline): skipped
      row.clear();
      return CTR_OK;
    }
    if (cols < 0) cols = (int32_t)row.size();
    if ((int32_t)row.size() != cols) {
      ::ctr::set_error("ctr_csv_to_bin: %s line %lld: %zu columns, expected %d", csv_path,
                       (long long)line, row.size(), cols);
      return CTR_ERR_INVALID;
    }
    wbuf.insert(wbuf.end(), row.begin(), row.end());
    if (wbuf.size() >= (1u << 20)) {
      if (fwrite(wbuf.data(), sizeof(int32_t), wbuf.size(), out.f) != wbuf.size()) {
        ::ctr::set_error("ctr_csv_to_bin: write failed");
        return CTR_ERR_INVALID;
      }
      wbuf.clear();
    }
    ++rows;
    row.clear();
    line_has_data = false;
    return CTR_OK;
  };
  size_t n;
  while ((n = fread(buf.data(), 1, buf.size(), in.f)) > 0) {
    for (size_t i = 0; i < n; ++i) {
      const char c = buf[i];
      if (c >= '0' && c <= '9') {
        if (!in_num) {
          in_num = true;
          neg = false;
          val = 0;
        }
        any_digit = true;
        val = val * 10 + (c - '0');
        if (val > (int64_t)INT32_MAX + 1) val = (int64_t)INT32_MAX + 2;  // saturate: error later
        line_has_data = true;
      } else if (c == ',') {
        if (!in_num || !end_token()) {
          ::ctr::set_error("ctr_csv_to_bin: %s line %lld: empty or bad field", csv_path,
                           (long long)line + 1);
          return CTR_ERR_INVALID;
        }
        line_has_data = true;
      } else if (c == '\n') {
        const int rc = end_line();
        if (rc != CTR_OK) return rc;
      } else if (c == '-' && !in_num) {
        in_num = true;
        neg = true;
        val = 0;
        line_has_data = true;
      } else if (c == '\r' || c == ' ' || c == '\t') {
        // CRLF line ends and padding around a field
      } else {
        ::ctr::set_error("ctr_csv_to_bin: %s line %lld: unexpected character 0x%02x", csv_path,
                         (long long)line + 1, (unsigned)(unsigned char)c);
        return CTR_ERR_INVALID;
      }
    }
  }
  CTR_REQUIRE(!ferror(in.f), "ctr_csv_to_bin: read error on %s", csv_path);
  if (line_has_data || in_num) {  // last line without a newline
    const int rc = end_line();
    if (rc != CTR_OK) return rc;
  }
  if (!wbuf.empty())
    CTR_REQUIRE(fwrite(wbuf.data(), sizeof(int32_t), wbuf.size(), out.f) == wbuf.size(),
                "ctr_csv_to_bin: write failed");
  h.rows = rows;
  h.cols = cols < 0 ? 0 : cols;
  CTR_REQUIRE(fseek(out.f, 0, SEEK_SET) == 0 && fwrite(&h, sizeof(h), 1, out.f) == 1,
              "ctr_csv_to_bin: header write failed");
  if (rows_out) *rows_out = h.rows;
  if (cols_out) *cols_out = h.cols;
  if (max_id_out) *max_id_out = h.max_id;
  return CTR_OK;
}

extern "C" int ctr_bin_info(const char* bin_path, int64_t* rows, int32_t* cols, int64_t* max_id,
                            int64_t* data_offset) {
  CTR_REQUIRE(bin_path, "ctr_bin_info: null path");
  File in;
  in.f = fopen(bin_path, "rb");
  CTR_REQUIRE(in.f, "ctr_bin_info: cannot open %s: %s", bin_path, strerror(errno));
  Header h;
  CTR_REQUIRE(fread(&h, sizeof(h), 1, in.f) == 1, "ctr_bin_info: %s: short header", bin_path);
  CTR_REQUIRE(memcmp(h.magic, kMagic, 8) == 0, "ctr_bin_info: %s: not a CTRBIN01 file", bin_path);
  CTR_REQUIRE(h.rows >= 0 && h.cols >= 0 && h.data_offset == kHeader,
              "ctr_bin_info: %s: corrupt header", bin_path);
  CTR_REQUIRE(fseek(in.f, 0, SEEK_END) == 0, "ctr_bin_info: seek failed");
  const long size = ftell(in.f);
  CTR_REQUIRE(size >= 0 && (int64_t)size == kHeader + h.rows * (int64_t)h.cols * 4,
              "ctr_bin_info: %s: size %ld does not match %lld x %d int32", bin_path, size,
              (long long)h.rows, h.cols);
  if (rows) *rows = h.rows;
  if (cols) *cols = h.cols;
  if (max_id) *max_id = h.max_id;
  if (data_offset) *data_offset = h.data_offset;
  return CTR_OK;
}
