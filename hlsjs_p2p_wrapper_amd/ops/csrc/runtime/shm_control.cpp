#include "shm_control.hpp"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <stdexcept>

#if defined(__x86_64__)
#include <immintrin.h>
#define HLSP2P_PAUSE() _mm_pause()
#else
#define HLSP2P_PAUSE() ((void)0)
#endif

namespace hlsp2p {

namespace {
constexpr uint64_t kMagic = 0x484c5350325043ull;  // "HLSP2PC"
}

ShmControl::ShmControl(const std::string& name, int rank, int world, int64_t slot_words, bool create)
    : name_(name), rank_(rank), world_(world), slot_words_(slot_words) {
  if (world < 1 || rank < 0 || rank >= world || slot_words < 1) throw std::invalid_argument("ShmControl: bad shape");
  if (name.empty() || name[0] != '/') throw std::invalid_argument("ShmControl: name must start with '/'");
  const size_t header = (sizeof(Header) + 63) / 64 * 64;
  bytes_ = header + sizeof(int64_t) * size_t(2) * size_t(world) * size_t(1 + slot_words);
  int fd = -1;
  if (create) {
    ::shm_unlink(name.c_str());  // a stale name from a killed run
    fd = ::shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("ShmControl: shm_open(create) failed for " + name);
    if (::ftruncate(fd, static_cast<off_t>(bytes_)) != 0) {
      ::close(fd);
      ::shm_unlink(name.c_str());
      throw std::runtime_error("ShmControl: ftruncate failed");
    }
  } else {
    fd = ::shm_open(name.c_str(), O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("ShmControl: shm_open(attach) failed for " + name);
    struct stat st;
    if (::fstat(fd, &st) != 0 || static_cast<size_t>(st.st_size) != bytes_) {
      ::close(fd);
      throw std::runtime_error("ShmControl: mapping size mismatch (world / slot_words differ across ranks?)");
    }
  }
  base_ = ::mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (base_ == MAP_FAILED) {
    base_ = nullptr;
    if (create) ::shm_unlink(name.c_str());
    throw std::runtime_error("ShmControl: mmap failed");
  }
  linked_ = create;
  hdr_ = static_cast<Header*>(base_);
  slots_ = reinterpret_cast<int64_t*>(static_cast<char*>(base_) + header);
  if (create) {
    // ftruncate zero-fills; publish the shape last so an attacher never sees a half header
    hdr_->world = world;
    hdr_->slot_words = slot_words;
    new (&hdr_->arrive) std::atomic<uint64_t>(0);
    std::atomic_thread_fence(std::memory_order_release);
    hdr_->magic = kMagic;
  } else if (hdr_->magic != kMagic || hdr_->world != world || hdr_->slot_words != slot_words) {
    ::munmap(base_, bytes_);
    base_ = nullptr;
    throw std::runtime_error("ShmControl: attached to a mapping of another shape");
  }
}

ShmControl::~ShmControl() {
  if (base_ != nullptr) ::munmap(base_, bytes_);
  if (linked_) ::shm_unlink(name_.c_str());
}

void ShmControl::unlink() {
  if (linked_) {
    ::shm_unlink(name_.c_str());
    linked_ = false;
  }
}

int64_t* ShmControl::slot(int parity, int r) const {
  return slots_ + (size_t(parity) * size_t(world_) + size_t(r)) * size_t(1 + slot_words_);
}

void ShmControl::arrive_and_wait(double timeout_s) {
  const uint64_t target = uint64_t(world_) * (gen_ + 1);
  hdr_->arrive.fetch_add(1, std::memory_order_acq_rel);  // release: our slot write
  // spin (pause) briefly, then yield: ranks are usually within microseconds of each
  // other, but an oversubscribed host must not burn the cores its peers need
  uint32_t spins = 0;
  auto t0 = std::chrono::steady_clock::now();
  while (hdr_->arrive.load(std::memory_order_acquire) < target) {
    if (++spins < 4096) {
      HLSP2P_PAUSE();
      continue;
    }
    sched_yield();
    if ((spins & 1023) == 0) {
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_s) throw std::runtime_error("ShmControl: timed out waiting for peers (a rank died?)");
    }
  }
  ++gen_;
}

void ShmControl::exchange(const int64_t* msg, int64_t n, double timeout_s) {
  int64_t* s = slot(static_cast<int>(gen_ & 1), rank_);
  if (n <= slot_words_ && n > 0) std::memcpy(s + 1, msg, sizeof(int64_t) * size_t(n));
  s[0] = n;
  arrive_and_wait(timeout_s);
}

void ShmControl::barrier(double timeout_s) { arrive_and_wait(timeout_s); }

int64_t ShmControl::length(int r) const {
  if (r < 0 || r >= world_) throw std::out_of_range("ShmControl: rank");
  return slot(static_cast<int>((gen_ - 1) & 1), r)[0];  // the generation just completed
}

void ShmControl::read(int r, int64_t* dst) const {
  const int64_t* s = slot(static_cast<int>((gen_ - 1) & 1), r);
  const int64_t n = s[0] < slot_words_ ? s[0] : slot_words_;
  if (n > 0) std::memcpy(dst, s + 1, sizeof(int64_t) * size_t(n));
}

}  // namespace hlsp2p
