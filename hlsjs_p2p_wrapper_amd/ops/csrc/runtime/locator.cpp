#include "locator.hpp"

namespace hlsp2p {

void SegmentLocator::add_dir(const std::string& dir, Dir d) { dirs_[dir] = std::move(d); }

int64_t SegmentLocator::resolve(const std::vector<std::string_view>& urls, int64_t* size, int64_t* ptr,
                                int64_t* base, int64_t* flags, uint8_t* ok) const {
  int64_t found = 0;
  std::string key;
  const Dir* last = nullptr;  // consecutive URLs usually share a directory
  std::string_view last_dir;
  for (size_t i = 0; i < urls.size(); ++i) {
    ok[i] = 0;
    size[i] = ptr[i] = base[i] = flags[i] = 0;
    const std::string_view u = urls[i];
    const size_t slash = u.rfind('/');
    if (slash == std::string_view::npos) continue;
    const std::string_view d = u.substr(0, slash + 1), name = u.substr(slash + 1);
    const Dir* e = nullptr;
    if (last != nullptr && d == last_dir) {
      e = last;
    } else {
      key.assign(d.data(), d.size());
      const auto it = dirs_.find(key);
      if (it == dirs_.end()) continue;
      e = &it->second;
      last = e;
      last_dir = d;
    }
    if (name.size() <= e->prefix.size() + e->suffix.size() || name.compare(0, e->prefix.size(), e->prefix) != 0 ||
        name.compare(name.size() - e->suffix.size(), e->suffix.size(), e->suffix) != 0)
      continue;
    const std::string_view digits = name.substr(e->prefix.size(), name.size() - e->prefix.size() - e->suffix.size());
    if (digits.size() > 18) continue;
    int64_t sn = 0;
    bool num = true;
    for (const char c : digits) {
      if (c < '0' || c > '9') {
        num = false;
        break;
      }
      sn = sn * 10 + (c - '0');
    }
    if (!num || sn < e->sn_lo || sn >= e->sn_hi || e->off.empty()) continue;
    const size_t slot = static_cast<size_t>(sn % static_cast<int64_t>(e->off.size()));
    size[i] = e->len[slot];
    ptr[i] = e->base + e->off[slot];
    base[i] = e->base;
    flags[i] = e->flags;
    ok[i] = 1;
    ++found;
  }
  return found;
}

}  // namespace hlsp2p
