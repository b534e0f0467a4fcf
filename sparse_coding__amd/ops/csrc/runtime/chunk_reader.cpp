// Native activation-chunk reader (host side of the HBM activation ring).
//
// Reference chunks are `torch.save`d fp16 tensors (activation_dataset.py:393-397):
// a zip archive whose "<name>/data/0" entry holds the raw storage bytes, stored
// uncompressed.  The reference reloads each 2 GiB chunk with torch.load (pickle
// + one big copy) before gathering batches on the CPU (big_sweep.py:401, :170).
// Here the zip central directory is parsed directly, the storage entry is read
// with parallel pread() calls into a caller-provided (pinned) host buffer by a
// small thread pool, asynchronously, so the next chunk streams from disk while
// the GPU trains on the current one.  No Python, no unpickling.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

uint16_t rd16(const unsigned char* p) { return p[0] | (p[1] << 8); }
uint32_t rd32(const unsigned char* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
uint64_t rd64(const unsigned char* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

bool pread_all(int fd, void* dst, size_t n, off_t off) {
  char* d = static_cast<char*>(dst);
  while (n > 0) {
    ssize_t r = pread(fd, d, n, off);
    if (r <= 0) return false;
    d += r;
    n -= (size_t)r;
    off += r;
  }
  return true;
}

// Find a stored (uncompressed) zip entry whose name ends with `suffix`.
// Returns 0 and the absolute data offset/size on success.
int zip_find(const char* path, const char* suffix, int64_t* out_off, int64_t* out_size) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) return -1;
  struct stat st;
  if (fstat(fd, &st) != 0) { close(fd); return -1; }
  const int64_t fsize = st.st_size;
  const int64_t tail = std::min<int64_t>(fsize, 65536 + 22);
  std::vector<unsigned char> buf(tail);
  if (!pread_all(fd, buf.data(), tail, fsize - tail)) { close(fd); return -2; }
  int64_t eocd = -1;
  for (int64_t i = tail - 22; i >= 0; --i)
    if (rd32(&buf[i]) == 0x06054b50) { eocd = i; break; }
  if (eocd < 0) { close(fd); return -3; }
  uint64_t cd_off = rd32(&buf[eocd + 16]);
  uint64_t cd_size = rd32(&buf[eocd + 12]);
  uint64_t n_entries = rd16(&buf[eocd + 10]);
  // zip64 end-of-central-directory locator (torch writes zip64 for big archives)
  if (eocd >= 20 && rd32(&buf[eocd - 20]) == 0x07064b50) {
    const uint64_t z64 = rd64(&buf[eocd - 20 + 8]);
    unsigned char zb[56];
    if (pread_all(fd, zb, 56, (off_t)z64) && rd32(zb) == 0x06064b50) {
      n_entries = rd64(zb + 32);
      cd_size = rd64(zb + 40);
      cd_off = rd64(zb + 48);
    }
  }
  std::vector<unsigned char> cd(cd_size);
  if (!pread_all(fd, cd.data(), cd_size, (off_t)cd_off)) { close(fd); return -4; }
  const size_t slen = strlen(suffix);
  size_t p = 0;
  for (uint64_t e = 0; e < n_entries && p + 46 <= cd.size(); ++e) {
    if (rd32(&cd[p]) != 0x02014b50) break;
    const uint16_t method = rd16(&cd[p + 10]);
    uint64_t csize = rd32(&cd[p + 20]), usize = rd32(&cd[p + 24]);
    const uint16_t nlen = rd16(&cd[p + 28]), xlen = rd16(&cd[p + 30]), clen = rd16(&cd[p + 32]);
    uint64_t loff = rd32(&cd[p + 42]);
    std::string name(reinterpret_cast<const char*>(&cd[p + 46]), nlen);
    // zip64 extra field
    size_t x = p + 46 + nlen, xend = x + xlen;
    while (x + 4 <= xend) {
      const uint16_t id = rd16(&cd[x]), sz = rd16(&cd[x + 2]);
      if (id == 0x0001) {
        size_t q = x + 4;
        if (usize == 0xFFFFFFFFu) { usize = rd64(&cd[q]); q += 8; }
        if (csize == 0xFFFFFFFFu) { csize = rd64(&cd[q]); q += 8; }
        if (loff == 0xFFFFFFFFu) { loff = rd64(&cd[q]); q += 8; }
      }
      x += 4 + sz;
    }
    if (name.size() >= slen && name.compare(name.size() - slen, slen, suffix) == 0) {
      if (method != 0) { close(fd); return -5; }  // compressed: not a torch.save archive
      unsigned char lh[30];
      if (!pread_all(fd, lh, 30, (off_t)loff) || rd32(lh) != 0x04034b50) { close(fd); return -6; }
      *out_off = (int64_t)loff + 30 + rd16(lh + 26) + rd16(lh + 28);
      *out_size = (int64_t)usize;
      close(fd);
      return 0;
    }
    p += 46 + nlen + xlen + clen;
  }
  close(fd);
  return -7;
}

struct Job {
  int ticket;
  std::string path;
  int64_t off, size;
  void* dst;
};

class Prefetcher {
 public:
  explicit Prefetcher(int nthreads) : stop_(false), next_(1) {
    for (int i = 0; i < std::max(1, nthreads); ++i) workers_.emplace_back([this] { run(); });
  }
  ~Prefetcher() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  // Split a read into ~32 MiB pieces so all workers share one big chunk.
  int submit(const char* path, int64_t off, int64_t size, void* dst) {
    const int64_t piece = 32ll << 20;
    std::lock_guard<std::mutex> g(mu_);
    const int ticket = next_++;
    int npieces = 0;
    for (int64_t o = 0; o < size; o += piece, ++npieces)
      queue_.push_back({ticket, path, off + o, std::min(piece, size - o), static_cast<char*>(dst) + o});
    pending_[ticket] = npieces;
    status_[ticket] = 0;
    cv_.notify_all();
    return ticket;
  }
  int wait(int ticket) {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_.count(ticket) == 0 || pending_[ticket] == 0; });
    const int s = status_[ticket];
    pending_.erase(ticket);
    status_.erase(ticket);
    return s;
  }
  int poll(int ticket) {
    std::lock_guard<std::mutex> g(mu_);
    return pending_.count(ticket) && pending_[ticket] > 0 ? 1 : 0;
  }

 private:
  void run() {
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !queue_.empty(); });
        if (stop_ && queue_.empty()) return;
        j = queue_.front();
        queue_.pop_front();
      }
      int fd = open(j.path.c_str(), O_RDONLY);
      bool ok = fd >= 0 && pread_all(fd, j.dst, (size_t)j.size, (off_t)j.off);
      if (fd >= 0) close(fd);
      {
        std::lock_guard<std::mutex> g(mu_);
        if (!ok) status_[j.ticket] = -1;
        if (--pending_[j.ticket] == 0) done_cv_.notify_all();
      }
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<Job> queue_;
  std::unordered_map<int, int> pending_, status_;
  std::vector<std::thread> workers_;
  bool stop_;
  int next_;
};

}  // namespace

extern "C" {

int sc_zip_find(const char* path, const char* suffix, int64_t* off, int64_t* size) {
  return zip_find(path, suffix, off, size);
}

void* sc_prefetcher_create(int nthreads) { return new Prefetcher(nthreads); }
void sc_prefetcher_destroy(void* p) { delete static_cast<Prefetcher*>(p); }
int sc_prefetch_submit(void* p, const char* path, int64_t off, int64_t size, void* dst) {
  return static_cast<Prefetcher*>(p)->submit(path, off, size, dst);
}
int sc_prefetch_wait(void* p, int ticket) { return static_cast<Prefetcher*>(p)->wait(ticket); }
int sc_prefetch_poll(void* p, int ticket) { return static_cast<Prefetcher*>(p)->poll(ticket); }

}  // extern "C"
