// RecordIO reader/writer (see recordio.h).
#include "recordio.h"

#include <cstring>
#include <stdexcept>

namespace mxamd {

namespace {
inline uint32_t EncodeLRec(uint32_t cflag, uint32_t len) { return (cflag << 29U) | len; }
inline uint32_t DecodeFlag(uint32_t rec) { return (rec >> 29U) & 7U; }
inline uint32_t DecodeLength(uint32_t rec) { return rec & ((1U << 29U) - 1U); }
}  // namespace

RecordWriter::RecordWriter(const std::string& path, bool append) {
  fp_ = std::fopen(path.c_str(), append ? "ab" : "wb");
  if (!fp_) throw std::runtime_error("cannot open " + path + " for writing");
}

RecordWriter::~RecordWriter() { Close(); }

void RecordWriter::Close() {
  if (fp_) {
    std::fclose(fp_);
    fp_ = nullptr;
  }
}

uint64_t RecordWriter::Tell() { return static_cast<uint64_t>(std::ftell(fp_)); }

uint64_t RecordWriter::Write(const char* buf, size_t size) {
  if (!fp_) throw std::runtime_error("RecordWriter is closed");
  if (size >= (1U << 29U)) throw std::runtime_error("RecordIO only accepts records < 512MB");
  uint64_t start = Tell();
  const uint32_t magic = kRecMagic;
  uint32_t len = static_cast<uint32_t>(size);
  uint32_t lower_align = (len >> 2U) << 2U;
  uint32_t upper_align = ((len + 3U) >> 2U) << 2U;
  uint32_t dptr = 0;
  for (uint32_t i = 0; i < lower_align; i += 4) {
    uint32_t w;
    std::memcpy(&w, buf + i, 4);
    if (w == magic) {
      uint32_t lrec = EncodeLRec(dptr == 0 ? 1U : 2U, i - dptr);
      std::fwrite(&magic, 4, 1, fp_);
      std::fwrite(&lrec, 4, 1, fp_);
      if (i != dptr) std::fwrite(buf + dptr, 1, i - dptr, fp_);
      dptr = i + 4;
    }
  }
  uint32_t lrec = EncodeLRec(dptr != 0 ? 3U : 0U, len - dptr);
  std::fwrite(&magic, 4, 1, fp_);
  std::fwrite(&lrec, 4, 1, fp_);
  if (len != dptr) std::fwrite(buf + dptr, 1, len - dptr, fp_);
  uint32_t zero = 0;
  if (upper_align != len) std::fwrite(&zero, 1, upper_align - len, fp_);
  return start;
}

RecordReader::RecordReader(const std::string& path) {
  fp_ = std::fopen(path.c_str(), "rb");
  if (!fp_) throw std::runtime_error("cannot open " + path + " for reading");
}

RecordReader::~RecordReader() { Close(); }

void RecordReader::Close() {
  if (fp_) {
    std::fclose(fp_);
    fp_ = nullptr;
  }
}

void RecordReader::Seek(uint64_t pos) { std::fseek(fp_, static_cast<long>(pos), SEEK_SET); }

uint64_t RecordReader::Tell() { return static_cast<uint64_t>(std::ftell(fp_)); }

bool RecordReader::Next(std::string* out) {
  out->clear();
  for (;;) {
    uint32_t header[2];
    size_t n = std::fread(header, 4, 2, fp_);
    if (n == 0) return false;
    if (n != 2) throw std::runtime_error("invalid RecordIO file (truncated header)");
    if (header[0] != kRecMagic) throw std::runtime_error("invalid RecordIO file (bad magic)");
    uint32_t cflag = DecodeFlag(header[1]);
    uint32_t len = DecodeLength(header[1]);
    uint32_t upper = ((len + 3U) >> 2U) << 2U;
    size_t base = out->size();
    out->resize(base + upper);
    if (upper && std::fread(&(*out)[base], 1, upper, fp_) != upper)
      throw std::runtime_error("invalid RecordIO file (truncated record)");
    out->resize(base + len);
    if (cflag == 0U || cflag == 3U) return true;
    const uint32_t magic = kRecMagic;
    out->append(reinterpret_cast<const char*>(&magic), 4);
  }
}

RecordPrefetcher::RecordPrefetcher(const std::string& path, std::vector<uint64_t> offsets,
                                   size_t capacity)
    : path_(path), offsets_(std::move(offsets)), capacity_(capacity ? capacity : 1) {
  th_ = std::thread([this] { Run(); });
}

RecordPrefetcher::~RecordPrefetcher() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

void RecordPrefetcher::Run() {
  try {
    RecordReader r(path_);
    for (uint64_t off : offsets_) {
      std::string rec;
      r.Seek(off);
      if (!r.Next(&rec)) break;
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return stop_ || q_.size() < capacity_; });
      if (stop_) return;
      q_.push_back(std::move(rec));
      cv_.notify_all();
    }
  } catch (...) {
  }
  std::lock_guard<std::mutex> lk(mu_);
  done_ = true;
  cv_.notify_all();
}

bool RecordPrefetcher::Next(std::string* out) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [this] { return !q_.empty() || done_; });
  if (q_.empty()) return false;
  *out = std::move(q_.front());
  q_.pop_front();
  cv_.notify_all();
  return true;
}

}  // namespace mxamd
