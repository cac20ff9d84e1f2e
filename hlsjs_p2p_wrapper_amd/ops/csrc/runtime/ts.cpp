#include "ts.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace hlsp2p {
namespace ts {
namespace {

constexpr int kPmtPidC = 0x1000;
constexpr int kVideoPidC = 0x100;
constexpr int kAudioPidC = 0x101;
constexpr int kId3PidC = 0x102;
constexpr int64_t kPtsBase = 900000;  // 10 s: streams rarely start at PTS 0

struct Rng {  // splitmix64
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  // bytes in [1, 255]: never 0, so random payload never forms a 00 00 01 start code
  void fill_nonzero(uint8_t* p, size_t n) {
    size_t i = 0;
    while (i < n) {
      uint64_t r = next();
      for (int k = 0; k < 8 && i < n; ++k, r >>= 8) p[i++] = static_cast<uint8_t>(1 + (r & 0xff) % 255);
    }
  }
};

struct PesUnit {
  int cls;  // 0 video, 1 audio, 2 id3
  int64_t dts;
  int64_t pts;
  bool has_dts;
  bool random_access;
  std::vector<uint8_t> es;
};

void put_ts(uint8_t* p, int marker, int64_t v) {
  v &= (int64_t(1) << 33) - 1;
  p[0] = static_cast<uint8_t>((marker << 4) | (((v >> 30) & 0x07) << 1) | 1);
  p[1] = static_cast<uint8_t>((v >> 22) & 0xff);
  p[2] = static_cast<uint8_t>((((v >> 15) & 0x7f) << 1) | 1);
  p[3] = static_cast<uint8_t>((v >> 7) & 0xff);
  p[4] = static_cast<uint8_t>(((v & 0x7f) << 1) | 1);
}

std::vector<uint8_t> pes_bytes(const PesUnit& u) {
  static const uint8_t sid[3] = {0xE0, 0xC0, 0xBD};
  const int hdr_data = u.has_dts ? 10 : 5;
  std::vector<uint8_t> out(9 + hdr_data + u.es.size());
  out[0] = 0; out[1] = 0; out[2] = 1;
  out[3] = sid[u.cls];
  size_t plen = 3 + hdr_data + u.es.size();
  if (u.cls == 0 && plen > 0xffff) plen = 0;  // unbounded video PES
  out[4] = static_cast<uint8_t>(plen >> 8);
  out[5] = static_cast<uint8_t>(plen & 0xff);
  out[6] = 0x80;
  out[7] = u.has_dts ? 0xC0 : 0x80;
  out[8] = static_cast<uint8_t>(hdr_data);
  put_ts(&out[9], u.has_dts ? 3 : 2, u.pts);
  if (u.has_dts) put_ts(&out[14], 1, u.dts);
  std::memcpy(&out[9 + hdr_data], u.es.data(), u.es.size());
  return out;
}

class Packetizer {
 public:
  std::vector<uint8_t> out;
  int cc[0x2000] = {0};

  void packet(int pid, bool pusi, const uint8_t* payload, int n_payload, const uint8_t* af, int af_len) {
    // af: adaptation-field body (flags + optional fields) of af_len bytes, or af_len < 0
    // for none.  Short payloads are padded with adaptation-field stuffing (0xFF).
    uint8_t pkt[kPacket];
    uint8_t body[184];
    int body_len = -1;
    if (af_len >= 0) {
      std::memcpy(body, af, af_len);
      body_len = af_len;
    }
    const int stuffing = 184 - (af_len >= 0 ? 1 + af_len : 0) - n_payload;
    if (stuffing > 0) {
      if (body_len < 0) {
        if (stuffing == 1) {
          body_len = 0;
        } else {
          body[0] = 0x00;
          std::memset(body + 1, 0xff, stuffing - 2);
          body_len = stuffing - 1;
        }
      } else {
        std::memset(body + body_len, 0xff, stuffing);
        body_len += stuffing;
      }
    }
    const int afc = (body_len >= 0 ? 2 : 0) | (n_payload > 0 ? 1 : 0);
    pkt[0] = 0x47;
    pkt[1] = static_cast<uint8_t>((pusi ? 0x40 : 0) | ((pid >> 8) & 0x1f));
    pkt[2] = static_cast<uint8_t>(pid & 0xff);
    pkt[3] = static_cast<uint8_t>((afc << 4) | (cc[pid] & 0x0f));
    if (afc & 1) cc[pid] = (cc[pid] + 1) & 0x0f;
    int pos = 4;
    if (body_len >= 0) {
      pkt[pos++] = static_cast<uint8_t>(body_len);
      std::memcpy(pkt + pos, body, body_len);
      pos += body_len;
    }
    std::memcpy(pkt + pos, payload, n_payload);
    out.insert(out.end(), pkt, pkt + kPacket);
  }

  void psi(int pid, const std::vector<uint8_t>& section) {
    std::vector<uint8_t> pl(1 + section.size());
    pl[0] = 0;  // pointer_field
    std::memcpy(pl.data() + 1, section.data(), section.size());
    uint8_t buf[184];
    std::memset(buf, 0xff, sizeof buf);
    std::memcpy(buf, pl.data(), pl.size());
    packet(pid, true, buf, 184, nullptr, -1);
  }

  void pes(int pid, const std::vector<uint8_t>& data, bool random_access, int64_t pcr) {
    size_t off = 0;
    bool first = true;
    while (off < data.size() || first) {
      uint8_t af[7];
      int af_len = -1;
      if (first && random_access) {
        af[0] = 0x50;  // random_access_indicator | PCR_flag
        int64_t base = pcr & ((int64_t(1) << 33) - 1);
        af[1] = static_cast<uint8_t>(base >> 25);
        af[2] = static_cast<uint8_t>(base >> 17);
        af[3] = static_cast<uint8_t>(base >> 9);
        af[4] = static_cast<uint8_t>(base >> 1);
        af[5] = static_cast<uint8_t>(((base & 1) << 7) | 0x7e);
        af[6] = 0;
        af_len = 7;
      }
      int room = 184 - (af_len >= 0 ? 1 + af_len : 0);
      int take = static_cast<int>(std::min<size_t>(room, data.size() - off));
      packet(pid, first, data.data() + off, take, af_len >= 0 ? af : nullptr, af_len);
      off += take;
      first = false;
    }
  }
};

std::vector<uint8_t> pat_section() {
  std::vector<uint8_t> s = {0x00, 0xB0, 0x00, 0x00, 0x01, 0xC1, 0x00, 0x00,
                            0x00, 0x01, static_cast<uint8_t>(0xE0 | (kPmtPidC >> 8)), static_cast<uint8_t>(kPmtPidC & 0xff)};
  int section_length = static_cast<int>(s.size()) - 3 + 4;
  s[1] = static_cast<uint8_t>(0xB0 | ((section_length >> 8) & 0x0f));
  s[2] = static_cast<uint8_t>(section_length & 0xff);
  uint32_t crc = mpeg_crc32(s.data(), s.size());
  for (int i = 3; i >= 0; --i) s.push_back(static_cast<uint8_t>(crc >> (8 * i)));
  return s;
}

std::vector<uint8_t> pmt_section(bool with_id3) {
  std::vector<uint8_t> s = {0x02, 0xB0, 0x00, 0x00, 0x01, 0xC1, 0x00, 0x00,
                            static_cast<uint8_t>(0xE0 | (kVideoPidC >> 8)), static_cast<uint8_t>(kVideoPidC & 0xff),
                            0xF0, 0x00};
  auto add = [&](int type, int pid) {
    s.push_back(static_cast<uint8_t>(type));
    s.push_back(static_cast<uint8_t>(0xE0 | (pid >> 8)));
    s.push_back(static_cast<uint8_t>(pid & 0xff));
    s.push_back(0xF0);
    s.push_back(0x00);
  };
  add(0x1B, kVideoPidC);
  add(0x0F, kAudioPidC);
  if (with_id3) add(0x15, kId3PidC);
  int section_length = static_cast<int>(s.size()) - 3 + 4;
  s[1] = static_cast<uint8_t>(0xB0 | ((section_length >> 8) & 0x0f));
  s[2] = static_cast<uint8_t>(section_length & 0xff);
  uint32_t crc = mpeg_crc32(s.data(), s.size());
  for (int i = 3; i >= 0; --i) s.push_back(static_cast<uint8_t>(crc >> (8 * i)));
  return s;
}

inline int64_t read_pts(const uint8_t* p) {
  return (int64_t((p[0] >> 1) & 0x07) << 30) | (int64_t(p[1]) << 22) | (int64_t(p[2] >> 1) << 15) |
         (int64_t(p[3]) << 7) | int64_t(p[4] >> 1);
}

}  // namespace

uint32_t mpeg_crc32(const uint8_t* p, size_t n) {
  uint32_t crc = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) {
    crc ^= uint32_t(p[i]) << 24;
    for (int k = 0; k < 8; ++k) crc = (crc & 0x80000000u) ? (crc << 1) ^ 0x04C11DB7u : (crc << 1);
  }
  return crc;
}

std::vector<uint8_t> mux_segment(const MuxConfig& cfg, MuxStats* stats) {
  Rng rng(cfg.seed * 0x100000001B3ull ^ uint64_t(cfg.sn) * 0x9E3779B97F4A7C15ull);
  const int nframes = std::max(1, static_cast<int>(std::lround(cfg.duration * cfg.fps)));
  const int64_t frame_ticks = static_cast<int64_t>(std::llround(90000.0 / cfg.fps));
  const int64_t t0 = kPtsBase + static_cast<int64_t>(std::llround(cfg.start_time * 90000.0));

  // ---- audio: ADTS AAC-LC 48 kHz stereo, 1024 samples/frame, 6 frames per PES
  const int n_aframes = std::max(1, static_cast<int>(cfg.duration * 48000.0 / 1024.0));
  const int64_t aframe_bytes = std::max<int64_t>(16, int64_t(cfg.audio_kbps) * 1000 / 8 * 1024 / 48000);
  std::vector<PesUnit> units;
  for (int f0 = 0; f0 < n_aframes; f0 += 6) {
    PesUnit u{1, 0, 0, false, false, {}};
    u.pts = t0 + static_cast<int64_t>(std::llround(f0 * 1024.0 * 90000.0 / 48000.0));
    u.dts = u.pts;
    for (int f = f0; f < std::min(n_aframes, f0 + 6); ++f) {
      int64_t len = aframe_bytes + 7;
      uint8_t h[7] = {0xFF, 0xF1, static_cast<uint8_t>((1 << 6) | (3 << 2) | (2 >> 2)),
                      static_cast<uint8_t>(((2 & 3) << 6) | ((len >> 11) & 0x03)),
                      static_cast<uint8_t>((len >> 3) & 0xff), static_cast<uint8_t>(((len & 7) << 5) | 0x1F), 0xFC};
      u.es.insert(u.es.end(), h, h + 7);
      size_t o = u.es.size();
      u.es.resize(o + aframe_bytes);
      rng.fill_nonzero(u.es.data() + o, aframe_bytes);
    }
    units.push_back(std::move(u));
  }
  int64_t audio_ts_bytes = 0;
  for (auto& u : units) audio_ts_bytes += (int64_t(u.es.size()) + 14 + 183) / 184 * kPacket;

  // ---- video: size the frames so the whole segment lands near target_bytes
  int64_t psi_bytes = 2 * kPacket;
  int64_t id3_bytes = cfg.with_id3 ? kPacket : 0;
  int64_t video_ts_budget = std::max<int64_t>(cfg.target_bytes - audio_ts_bytes - psi_bytes - id3_bytes,
                                              int64_t(nframes) * kPacket);
  int64_t video_es_budget = video_ts_budget * 184 / kPacket - int64_t(nframes) * (19 + 96);
  std::vector<double> w(nframes);
  double wsum = 0;
  for (int f = 0; f < nframes; ++f) {
    w[f] = (f == 0 ? 8.0 : 1.0) * (0.8 + 0.4 * rng.uniform());
    wsum += w[f];
  }
  for (int f = 0; f < nframes; ++f) {
    PesUnit u{0, 0, 0, true, f == 0, {}};
    u.dts = t0 + int64_t(f) * frame_ticks;
    u.pts = u.dts + frame_ticks;  // one frame of composition delay
    int64_t sz = std::max<int64_t>(64, static_cast<int64_t>(video_es_budget * (w[f] / wsum)));
    static const uint8_t aud[6] = {0, 0, 0, 1, 0x09, 0xF0};
    u.es.insert(u.es.end(), aud, aud + 6);
    if (f == 0) {
      uint8_t sps[5] = {0, 0, 0, 1, 0x67};
      u.es.insert(u.es.end(), sps, sps + 5);
      size_t o = u.es.size();
      u.es.resize(o + 10);
      rng.fill_nonzero(u.es.data() + o, 10);
      uint8_t pps[5] = {0, 0, 0, 1, 0x68};
      u.es.insert(u.es.end(), pps, pps + 5);
      o = u.es.size();
      u.es.resize(o + 4);
      rng.fill_nonzero(u.es.data() + o, 4);
    }
    uint8_t slice[5] = {0, 0, 0, 1, static_cast<uint8_t>(f == 0 ? 0x65 : 0x41)};
    u.es.insert(u.es.end(), slice, slice + 5);
    size_t o = u.es.size();
    int64_t body = std::max<int64_t>(16, sz - int64_t(o));
    u.es.resize(o + body);
    rng.fill_nonzero(u.es.data() + o, body);
    units.push_back(std::move(u));
  }
  if (cfg.with_id3) {
    PesUnit u{2, t0, t0, false, false, {}};
    const char tag[] = "ID3\x04\x00\x00\x00\x00\x00\x10PRIV\x00\x00\x00\x06\x00\x00hlsp2p";
    u.es.assign(tag, tag + sizeof(tag) - 1);
    units.push_back(std::move(u));
  }
  std::stable_sort(units.begin(), units.end(), [](const PesUnit& a, const PesUnit& b) {
    if (a.dts != b.dts) return a.dts < b.dts;
    return a.cls < b.cls;
  });

  Packetizer pk;
  pk.out.reserve(static_cast<size_t>(cfg.target_bytes) + 64 * kPacket);
  pk.psi(0, pat_section());
  pk.psi(kPmtPidC, pmt_section(cfg.with_id3));
  static const int pids[3] = {kVideoPidC, kAudioPidC, kId3PidC};
  MuxStats st;
  for (const PesUnit& u : units) {
    std::vector<uint8_t> pes = pes_bytes(u);
    pk.pes(pids[u.cls], pes, u.random_access, u.dts - 9000);
    st.es_bytes[u.cls] += int64_t(u.es.size());
    st.n_pes[u.cls] += 1;
    if (st.first_pts[u.cls] < 0) st.first_pts[u.cls] = u.pts;
    st.last_pts[u.cls] = std::max(st.last_pts[u.cls], u.pts);
  }
  st.n_packets = int64_t(pk.out.size() / kPacket);
  if (stats) *stats = st;
  return std::move(pk.out);
}

void demux_segment(const uint8_t* data, int64_t n, uint8_t* es_out, int64_t* pes_out, int64_t max_pes, int64_t* info) {
  std::fill(info, info + kInfoWords, 0);
  for (int64_t i = 0; i < int64_t(kClasses) * max_pes * 3; ++i) pes_out[i] = -1;
  int64_t status = 0;
  const int64_t np = n / kPacket;
  if (n % kPacket) status |= kBadLength;
  info[kNumPackets] = np;
  // --- PSI: PAT then PMT within the first kPsiScanPackets packets
  int pmt_pid = -1, vpid = -1, apid = -1, ipid = -1, vtype = 0, atype = 0;
  const int64_t scan = std::min<int64_t>(np, kPsiScanPackets);
  for (int64_t i = 0; i < scan && pmt_pid < 0; ++i) {
    const uint8_t* p = data + i * kPacket;
    if (p[0] != 0x47) continue;
    int pid = ((p[1] & 0x1f) << 8) | p[2];
    if (pid != 0 || !(p[1] & 0x40)) continue;
    int afc = (p[3] >> 4) & 3;
    int ps = 4 + ((afc & 2) ? 1 + p[4] : 0);
    if (!(afc & 1) || ps >= kPacket) continue;
    ps += 1 + p[ps];  // pointer field
    if (ps + 8 > kPacket || p[ps] != 0x00) continue;
    int slen = ((p[ps + 1] & 0x0f) << 8) | p[ps + 2];
    int end = std::min(ps + 3 + slen - 4, kPacket);
    for (int q = ps + 8; q + 4 <= end; q += 4) {
      int prog = (p[q] << 8) | p[q + 1];
      if (prog != 0) { pmt_pid = ((p[q + 2] & 0x1f) << 8) | p[q + 3]; break; }
    }
  }
  if (pmt_pid < 0) status |= kNoPat;
  bool pmt_found = false;
  for (int64_t i = 0; i < scan && pmt_pid >= 0 && !pmt_found; ++i) {
    const uint8_t* p = data + i * kPacket;
    if (p[0] != 0x47) continue;
    int pid = ((p[1] & 0x1f) << 8) | p[2];
    if (pid != pmt_pid || !(p[1] & 0x40)) continue;
    int afc = (p[3] >> 4) & 3;
    int ps = 4 + ((afc & 2) ? 1 + p[4] : 0);
    if (!(afc & 1) || ps >= kPacket) continue;
    ps += 1 + p[ps];
    if (ps + 12 > kPacket || p[ps] != 0x02) continue;
    pmt_found = true;
    int slen = ((p[ps + 1] & 0x0f) << 8) | p[ps + 2];
    int end = std::min(ps + 3 + slen - 4, kPacket);
    int pil = ((p[ps + 10] & 0x0f) << 8) | p[ps + 11];
    for (int q = ps + 12 + pil; q + 5 <= end;) {
      int type = p[q];
      int epid = ((p[q + 1] & 0x1f) << 8) | p[q + 2];
      int eil = ((p[q + 3] & 0x0f) << 8) | p[q + 4];
      if ((type == 0x1B || type == 0x24) && vpid < 0) { vpid = epid; vtype = type; }
      else if ((type == 0x0F || type == 0x03 || type == 0x04) && apid < 0) { apid = epid; atype = type; }
      else if (type == 0x15 && ipid < 0) { ipid = epid; }
      q += 5 + eil;
    }
  }
  if (pmt_pid >= 0 && !pmt_found) status |= kNoPmt;
  info[kPmtPid] = pmt_pid; info[kVideoPid] = vpid; info[kAudioPid] = apid; info[kId3Pid] = ipid;
  info[kVideoType] = vtype; info[kAudioType] = atype;
  const int cls_pid[3] = {vpid, apid, ipid};
  // --- two passes: sizes, then copy
  int64_t bytes[kClasses] = {0, 0, 0};
  int64_t npes[kClasses] = {0, 0, 0};
  int64_t first_pts[kClasses] = {-1, -1, -1};
  int64_t last_pts[kClasses] = {-1, -1, -1};
  for (int pass = 0; pass < 2; ++pass) {
    int64_t base[kClasses] = {0, bytes[0], bytes[0] + bytes[1]};
    int64_t cur[kClasses] = {0, 0, 0};
    int64_t cnt[kClasses] = {0, 0, 0};
    for (int64_t i = 0; i < np; ++i) {
      const uint8_t* p = data + i * kPacket;
      if (p[0] != 0x47) { if (pass == 0) status |= kBadSync; continue; }
      int pid = ((p[1] & 0x1f) << 8) | p[2];
      int c = -1;
      for (int k = 0; k < kClasses; ++k) if (cls_pid[k] >= 0 && pid == cls_pid[k]) { c = k; break; }
      if (c < 0) continue;
      int afc = (p[3] >> 4) & 3;
      if (!(afc & 1)) continue;
      int ps = 4 + ((afc & 2) ? 1 + p[4] : 0);
      if (ps > kPacket) { if (pass == 0) status |= kBadLength; continue; }
      int len = kPacket - ps;
      if (p[1] & 0x40) {
        const uint8_t* h = p + ps;
        if (len < 9 || h[0] != 0 || h[1] != 0 || h[2] != 1 || 9 + h[8] > len) {
          if (pass == 0) status |= kPesHeaderError;
          continue;
        }
        int64_t pts = -1, dts = -1;
        if ((h[7] & 0x80) && len >= 14) pts = read_pts(h + 9);
        if ((h[7] & 0xC0) == 0xC0 && len >= 19) dts = read_pts(h + 14);
        if (pass == 1) {
          if (cnt[c] == 0) first_pts[c] = pts;
          last_pts[c] = pts;
          if (cnt[c] < max_pes) {
            int64_t* r = pes_out + (int64_t(c) * max_pes + cnt[c]) * 3;
            r[0] = cur[c]; r[1] = pts; r[2] = dts;
          }
        }
        cnt[c] += 1;
        int skip = 9 + h[8];
        ps += skip;
        len -= skip;
      }
      if (pass == 1 && len > 0) std::memcpy(es_out + base[c] + cur[c], p + ps, len);
      cur[c] += len;
    }
    if (pass == 0) { for (int k = 0; k < kClasses; ++k) { bytes[k] = cur[k]; npes[k] = cnt[k]; } }
  }
  for (int k = 0; k < kClasses; ++k) {
    info[kVideoBytes + k] = bytes[k];
    info[kNumVideoPes + k] = npes[k];
    info[kFirstPts + k] = -1;
    info[kLastPts + k] = -1;
    if (npes[k] > max_pes) status |= kPesOverflow;
  }
  for (int k = 0; k < kClasses; ++k) {  // first / last PES PTS (recorded in pass 1)
    if (npes[k] > 0) info[kFirstPts + k] = first_pts[k];
    if (npes[k] > 0) info[kLastPts + k] = last_pts[k];
  }
  info[kPayloadBytes] = bytes[0] + bytes[1] + bytes[2];
  info[kAudioEsOffset] = bytes[0];
  info[kId3EsOffset] = bytes[0] + bytes[1];
  info[kStatus] = status;
}

}  // namespace ts
}  // namespace hlsp2p
