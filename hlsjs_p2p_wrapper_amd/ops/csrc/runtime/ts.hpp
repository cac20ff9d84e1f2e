// MPEG-2 Transport Stream: synthetic muxer (origin packager) and the CPU reference
// demuxer whose output format the CDNA4 demux kernels (kernels/ts_demux.hip) reproduce
// byte-for-byte.
//
// In the reference the TS demux happens inside hls.js after FRAG_LOADED (its use is
// evidenced by the demuxer monkey-patch in test/hls-controllers.js:60-62); SURVEY §2.2 K11
// moves it on-device.  Scope is the TS layer: 188-byte packet sync, PAT/PMT, PID filter
// into video/audio/ID3 classes, PES reassembly with PTS/DTS.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace hlsp2p {
namespace ts {

constexpr int kPacket = 188;
constexpr int kPsiScanPackets = 64;  // PAT/PMT must appear within the first 64 packets
constexpr int kClasses = 3;          // 0 video, 1 audio, 2 id3/metadata
constexpr int kInfoWords = 24;

// info[] layout (int64), identical on host and device
enum Info : int {
  kStatus = 0,
  kPmtPid = 1,
  kVideoPid = 2,
  kAudioPid = 3,
  kId3Pid = 4,
  kNumPackets = 5,
  kVideoBytes = 6,   // kVideoBytes + class
  kNumVideoPes = 9,  // kNumVideoPes + class
  kVideoType = 12,
  kAudioType = 13,
  kPayloadBytes = 14,  // total ES bytes (video+audio+id3)
  kFirstPts = 16,      // kFirstPts + class: PTS of the class's first PES (-1 if none)
  kLastPts = 19,       // kLastPts + class: PTS of the class's last PES
  kAudioEsOffset = 22,  // byte offset of the audio ES from the segment's ES start (video at 0)
  kId3EsOffset = 23,    // byte offset of the id3 ES (the host and the split kernels pack
                        // [video | audio | id3]; the fused kernel uses fixed per-class regions)
};
// status bits
enum Status : int64_t {
  kBadSync = 1,
  kNoPat = 2,
  kNoPmt = 4,
  kPesOverflow = 8,
  kPesHeaderError = 16,
  kBadLength = 32,
};

struct MuxConfig {
  double duration = 4.0;
  double fps = 25.0;
  int64_t target_bytes = 3000000;
  int audio_kbps = 128;
  bool with_id3 = false;
  uint64_t seed = 1;
  int64_t sn = 0;
  double start_time = 0.0;
};

struct MuxStats {
  int64_t es_bytes[kClasses] = {0, 0, 0};
  int64_t n_pes[kClasses] = {0, 0, 0};
  int64_t first_pts[kClasses] = {-1, -1, -1};
  int64_t last_pts[kClasses] = {-1, -1, -1};
  int64_t n_packets = 0;
};

std::vector<uint8_t> mux_segment(const MuxConfig& cfg, MuxStats* stats);

// CPU reference demux of one segment.
//   es_out:  >= n bytes; receives [video ES | audio ES | id3 ES]
//   pes_out: int64[kClasses][max_pes][3] = (es_offset, pts, dts), -1 when absent
//   info:    int64[kInfoWords]
void demux_segment(const uint8_t* data, int64_t n, uint8_t* es_out, int64_t* pes_out, int64_t max_pes,
                   int64_t* info);

uint32_t mpeg_crc32(const uint8_t* p, size_t n);

}  // namespace ts
}  // namespace hlsp2p
