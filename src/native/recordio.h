// RecordIO container format (dmlc-core recordio; used by MXNet .rec files).
//
// Parity: 3rdparty/dmlc-core include/dmlc/recordio.h (kMagic 0xced7230a,
// lrec = cflag << 29 | length, 4-byte padding, records split at embedded
// magic words with cflag 1/2/3) and python/mxnet/recordio.py.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace mxamd {

constexpr uint32_t kRecMagic = 0xced7230a;

class RecordWriter {
 public:
  explicit RecordWriter(const std::string& path, bool append = false);
  ~RecordWriter();
  // returns the byte offset at which the record starts
  uint64_t Write(const char* buf, size_t size);
  uint64_t Tell();
  void Close();

 private:
  FILE* fp_ = nullptr;
};

class RecordReader {
 public:
  explicit RecordReader(const std::string& path);
  ~RecordReader();
  bool Next(std::string* out);  // false at EOF
  void Seek(uint64_t pos);
  uint64_t Tell();
  void Close();

 private:
  FILE* fp_ = nullptr;
};

// Background reader: fetches records at the given offsets (in order) on a
// worker thread into a bounded queue — the IO stage of ImageRecordIter.
class RecordPrefetcher {
 public:
  RecordPrefetcher(const std::string& path, std::vector<uint64_t> offsets, size_t capacity);
  ~RecordPrefetcher();
  bool Next(std::string* out);  // false when exhausted

 private:
  void Run();
  std::string path_;
  std::vector<uint64_t> offsets_;
  size_t capacity_;
  std::deque<std::string> q_;
  bool done_ = false, stop_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread th_;
};

}  // namespace mxamd
