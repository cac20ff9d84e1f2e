// Native URL -> CDN-bytes locator for origins whose segment bytes never move (a VOD origin's
// pinned-host or HBM pools).  The swarm node resolves every fragment request to (size,
// address, allocation base, want flags) before it becomes a want row; for the synthetic
// origins that is a path parse + a pool lookup in Python (~1 us per fragment on the rank,
// the largest single cost of the fleet rank's admission).  Here a batch of URLs is resolved
// in one call: the URL's directory is looked up in a hash map of registered segment
// directories, the file name "<prefix><sn><suffix>" is parsed, and the sequence number picks
// the pool slot (sn % pool).  URLs it does not know come back unresolved: the caller takes
// its general Python path for them (network origins, live windows, byte ranges, faults).
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace hlsp2p {

class SegmentLocator {
 public:
  struct Dir {
    std::string prefix, suffix;   // file name around the decimal sequence number
    int64_t sn_lo = 0, sn_hi = 0;  // served sequence numbers [sn_lo, sn_hi)
    int64_t base = 0;              // allocation base address of the pool
    int64_t flags = 0;             // want flags of every segment (e.g. on device)
    std::vector<int64_t> off, len;  // per pool slot
  };

  // Register (or replace) a segment directory: URLs "<dir><prefix><sn><suffix>".
  void add_dir(const std::string& dir, Dir d);
  // Resolve n URLs; ok[i] = 0 for those it does not serve.
  int64_t resolve(const std::vector<std::string_view>& urls, int64_t* size, int64_t* ptr, int64_t* base,
                  int64_t* flags, uint8_t* ok) const;
  void clear() { dirs_.clear(); }
  size_t size() const { return dirs_.size(); }

 private:
  std::unordered_map<std::string, Dir> dirs_;
};

}  // namespace hlsp2p
