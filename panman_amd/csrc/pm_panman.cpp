// pm_panman.cpp -- PanMAN file IO without the capnp library: xz (liblzma) + the standard
// (unpacked) Cap'n Proto wire format, for the schema in panman.capnp.
//
// Reader: TreeGroup(istream) + Tree::protoMATToTree + assignMutationsToNodes
//   (src/panman.cpp:6847-6877, :1661-1751, :576-618; NucMut / BlockMut from a reader:
//   src/panman.hpp:192-210, :441-452).  Multi-segment messages, far and double-far
//   pointers are followed; every offset is bounds-checked.
// Writer: TreeGroup::writeToFile + Tree::getNodesPreorder (src/panman.cpp:6885-7015,
//   :2854-2932), xz-compressed as writePanMAN does (src/panmanUtils.cpp:271-299).
//
// Struct layouts (data words, pointers) follow capnp's field allocation for panman.capnp:
//   NucMut(2,0): nucPosition i32@0 nucGapPosition i32@32 nucGapExist bit64 mutInfo u32@96
//   Mutation(2,1): blockId i64@0 blockGapExist bit64 blockMutExist bit65 blockMutInfo
//     bit66 blockInversion bit67; ptr0 nucMutation
//   Node(0,2) ConsensusSeqToBlockIds(0,4) GapList(2,2: blockId i64@0, blockGapExist bit64)
//   BlockGapList(0,2) CircularOffset / RotationIndex(1,1: i32@0) SequenceInverted(1,1: bit0)
//   Tree(0,8) TreeGroup(0,2) ComplexMutation(10,3)
// Old format (pm_panman_load_old): an xz-compressed Google Protobuf `panmanOld.treeGroup`
//   (panman.proto), read by TreeGroup(istream, isOld = true) + Tree::protoMATToTree(
//   panmanOld::tree) + assignMutationsToNodes (src/panman.cpp:6865-6876, :1803-1866,
//   :1773-1801; NucMut / BlockMut from panmanOld: src/panman.hpp:212-230, :454-465) and
//   converted by the commented-out CLI command --protobuf2capnp (src/panmanUtils.cpp:939-952).
//   Decoded by hand from the protobuf wire format (varint / 64-bit / length-delimited /
//   32-bit records; repeated scalars packed or not), into the same PanmanTree as a .panman.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <new>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "pm_internal.h"
#include "pm_newick.h"
#include "pm_panman_tree.h"

// ---- liblzma (linked as liblzma.so.5; prototypes of its stable C ABI) ----------------
extern "C" {
struct pm_lzma_stream {
    const uint8_t* next_in;
    size_t avail_in;
    uint64_t total_in;
    uint8_t* next_out;
    size_t avail_out;
    uint64_t total_out;
    const void* allocator;
    void* internal;
    void* reserved_ptr1;
    void* reserved_ptr2;
    void* reserved_ptr3;
    void* reserved_ptr4;
    uint64_t reserved_int1;
    uint64_t reserved_int2;
    size_t reserved_int3;
    size_t reserved_int4;
    int reserved_enum1;
    int reserved_enum2;
};
int lzma_stream_decoder(pm_lzma_stream* strm, uint64_t memlimit, uint32_t flags);
int lzma_easy_encoder(pm_lzma_stream* strm, uint32_t preset, int check);
// lzma_mt (liblzma >= 5.2): the multi-threaded .xz encoder's options
struct pm_lzma_mt {
    uint32_t flags;
    uint32_t threads;
    uint64_t block_size;
    uint32_t timeout;
    uint32_t preset;
    const void* filters;
    int check;
    int reserved_enum1, reserved_enum2, reserved_enum3;
    uint32_t reserved_int1, reserved_int2, reserved_int3, reserved_int4;
    uint64_t reserved_int5, reserved_int6, reserved_int7, reserved_int8;
    void *reserved_ptr1, *reserved_ptr2, *reserved_ptr3, *reserved_ptr4;
};
int lzma_stream_encoder_mt(pm_lzma_stream* strm, const pm_lzma_mt* options);
// lzma_filter, and the preset expansion into an lzma_options_lzma (whose first member is
// dict_size; the rest is filled by liblzma and passed back opaque)
struct pm_lzma_filter {
    uint64_t id;
    void* options;
};
unsigned char lzma_lzma_preset(void* options, uint32_t preset);
int lzma_stream_encoder(pm_lzma_stream* strm, const pm_lzma_filter* filters, int check);
int lzma_code(pm_lzma_stream* strm, int action);
void lzma_end(pm_lzma_stream* strm);
uint32_t lzma_crc32(const uint8_t* buf, size_t size, uint32_t crc);
}

namespace pm {
namespace {

constexpr int kLzmaOk = 0, kLzmaStreamEnd = 1, kLzmaFinish = 3, kLzmaCheckCrc64 = 4;
constexpr uint32_t kLzmaConcatenated = 0x08;

// Decoded messages: a byte vector whose resize leaves new bytes uninitialised (every byte is
// written by the decoder; zero-filling a C5-sized message first cost a single-threaded pass).
template <class T>
struct DefaultInit : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = DefaultInit<U>;
    };
    DefaultInit() = default;
    template <class U>
    DefaultInit(const DefaultInit<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept {
        ::new (static_cast<void*>(p)) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};
using Bytes = std::vector<uint8_t, DefaultInit<uint8_t>>;

bool xz_decode_serial(const std::vector<uint8_t>& in, Bytes& out, std::string& err);

// ---- multi-block .xz in parallel --------------------------------------------------------
// The writer (xz_encode) emits one stream of independent blocks; its index (at the end of the
// stream) gives every block's compressed and uncompressed size, so each block can be decoded
// on its own host thread: re-wrapped as a one-block stream (the original stream header, the
// block, a one-record index and a footer, CRCs by liblzma) and decoded into its slice of the
// output.  Anything else -- one block (what the reference writes), several streams, stream
// padding, a malformed index -- takes the single-threaded decoder.
struct XzBlock {
    size_t offset;       // in the input
    uint64_t unpadded;   // block header + data + check (index "unpadded size")
    uint64_t size;       // uncompressed
    size_t out;          // offset of its output
};

bool vli_read(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
    v = 0;
    for (int i = 0; i < 9 && p < end; ++i) {
        const uint8_t b = *p++;
        v |= (uint64_t)(b & 0x7f) << (7 * i);
        if (!(b & 0x80)) return i == 0 || b != 0;
    }
    return false;
}

void vli_write(std::vector<uint8_t>& o, uint64_t v) {
    while (v >= 0x80) {
        o.push_back((uint8_t)(v | 0x80));
        v >>= 7;
    }
    o.push_back((uint8_t)v);
}

uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
void wr32(std::vector<uint8_t>& o, uint32_t v) {
    for (int i = 0; i < 4; ++i) o.push_back((uint8_t)(v >> (8 * i)));
}

bool xz_blocks(const std::vector<uint8_t>& in, std::vector<XzBlock>& blocks) {
    const size_t n = in.size();
    if (n < 32 || in[n - 2] != 'Y' || in[n - 1] != 'Z') return false;
    const uint8_t* foot = in.data() + n - 12;
    if (lzma_crc32(foot + 4, 6, 0) != rd32(foot)) return false;
    if (foot[8] != in[6] || foot[9] != in[7]) return false;   // stream flags as in the header
    const uint64_t index_size = ((uint64_t)rd32(foot + 4) + 1) * 4;
    if (index_size + 24 > n) return false;
    const uint8_t* idx = foot - index_size;
    if (idx[0] != 0 || lzma_crc32(idx, index_size - 4, 0) != rd32(foot - 4)) return false;
    const uint8_t* p = idx + 1;
    uint64_t count = 0;
    if (!vli_read(p, foot - 4, count) || count < 2 || count > (1u << 20)) return false;
    // The index's sizes are attacker-controlled (its CRC is computable): every block must fit
    // between the stream header and the index, and the declared output must stay below a cap
    // (a generous multiple of the input; a legitimate stream beyond it still decodes, serially,
    // into a buffer grown from the data itself).  Nothing here can wrap: sizes are checked
    // against what remains before they are added.
    const uint64_t idx_pos = (uint64_t)(idx - in.data());
    const uint64_t out_cap = std::min<uint64_t>((uint64_t)n * 4096 + ((uint64_t)1 << 20), (uint64_t)1 << 42);
    uint64_t off = 12, out = 0;
    for (uint64_t k = 0; k < count; ++k) {
        XzBlock b{};
        if (!vli_read(p, foot - 4, b.unpadded) || !vli_read(p, foot - 4, b.size) || b.unpadded < 5) return false;
        const uint64_t padded = (b.unpadded + 3) & ~(uint64_t)3;   // (a VLI is < 2^63)
        if (padded > idx_pos - off || b.size > out_cap - out) return false;
        b.offset = (size_t)off;
        b.out = (size_t)out;
        off += padded;
        out += b.size;
        blocks.push_back(b);
    }
    return off == idx_pos;   // one stream: the blocks end where the index starts
}

bool xz_decode(const std::vector<uint8_t>& in, Bytes& out, std::string& err) {
    std::vector<XzBlock> blocks;
    if (!xz_blocks(in, blocks)) return xz_decode_serial(in, out, err);
    try {
        out.resize(blocks.back().out + (size_t)blocks.back().size);
    } catch (const std::bad_alloc&) {
        out.clear();
        return xz_decode_serial(in, out, err);
    }
    std::vector<int> ok(blocks.size(), 0);
    host_parallel_for((int)blocks.size(), [&](int k) {
        const XzBlock& b = blocks[(size_t)k];
        const size_t padded = (size_t)((b.unpadded + 3) & ~(uint64_t)3);
        std::vector<uint8_t> one(in.begin(), in.begin() + 12);   // stream header
        one.insert(one.end(), in.begin() + (ptrdiff_t)b.offset, in.begin() + (ptrdiff_t)(b.offset + padded));
        std::vector<uint8_t> index{0};
        vli_write(index, 1);
        vli_write(index, b.unpadded);
        vli_write(index, b.size);
        while (index.size() % 4) index.push_back(0);
        wr32(index, lzma_crc32(index.data(), index.size(), 0));
        one.insert(one.end(), index.begin(), index.end());
        std::vector<uint8_t> tail;
        wr32(tail, (uint32_t)(index.size() / 4 - 1));
        tail.push_back(in[6]);
        tail.push_back(in[7]);
        std::vector<uint8_t> foot;
        wr32(foot, lzma_crc32(tail.data(), tail.size(), 0));
        foot.insert(foot.end(), tail.begin(), tail.end());
        foot.push_back('Y');
        foot.push_back('Z');
        one.insert(one.end(), foot.begin(), foot.end());
        pm_lzma_stream s{};
        if (lzma_stream_decoder(&s, UINT64_MAX, 0) != kLzmaOk) return;
        s.next_in = one.data();
        s.avail_in = one.size();
        uint8_t extra = 0;
        s.next_out = b.size ? out.data() + b.out : &extra;
        s.avail_out = (size_t)b.size;
        int rc = lzma_code(&s, kLzmaFinish);
        if (rc == kLzmaOk && s.avail_out == 0) {   // the end of stream needs one more call
            s.next_out = &extra;
            s.avail_out = 1;
            rc = lzma_code(&s, kLzmaFinish);
            ok[(size_t)k] = rc == kLzmaStreamEnd && s.avail_out == 1;
        } else {
            ok[(size_t)k] = rc == kLzmaStreamEnd && s.avail_out == 0;
        }
        lzma_end(&s);
    });
    for (int v : ok)
        if (!v) return xz_decode_serial(in, out, err);   // (a block that does not decode alone)
    phase_add("panman.xz_parallel_blocks", (double)blocks.size());   // (a count, not seconds)
    return true;
}

bool xz_decode_serial(const std::vector<uint8_t>& in, Bytes& out, std::string& err) {
    pm_lzma_stream s{};
    if (lzma_stream_decoder(&s, UINT64_MAX, kLzmaConcatenated) != kLzmaOk) { err = "xz decoder init"; return false; }
    out.resize(std::max<size_t>(in.size() * 4, 1 << 20));
    s.next_in = in.data();
    s.avail_in = in.size();
    size_t done = 0;
    for (;;) {
        s.next_out = out.data() + done;
        s.avail_out = out.size() - done;
        const int rc = lzma_code(&s, kLzmaFinish);
        done = out.size() - s.avail_out;
        if (rc == kLzmaStreamEnd) break;
        if (rc != kLzmaOk) { lzma_end(&s); err = "xz data error " + std::to_string(rc); return false; }
        if (s.avail_out == 0) out.resize(out.size() * 2);
        else if (s.avail_in == 0) { lzma_end(&s); err = "truncated xz stream"; return false; }
    }
    lzma_end(&s);
    out.resize(done);
    return true;
}

// xz level 9 as writePanMAN (src/panmanUtils.cpp:282-285): the preset's LZMA2 settings
// (match finder, nice length, lc / lp / pb) with the dictionary cut to the data it can
// reach -- a dictionary larger than the input (or than one block) finds nothing more, but
// the level-9 encoder initialises all 64 MiB of it, which dominated writing a small PanMAN.
// Messages above one block go through liblzma's multi-threaded encoder in independent
// blocks whose size depends on the message size only (xz_block_size; the bytes written do
// not depend on the machine's core count): still one standard .xz stream that any xz decoder
// (the reference's boost lzma filter included) reads back to the same bytes.  Level 9 encodes
// PanMAN messages at ~2 MB/s a thread, so a message of a few hundred KiB (a 2 000-leaf PanMAN)
// is cut into >= 16 blocks of >= 64 KiB (+3-6 % of file size against one block), a large one
// into 1 MiB blocks.  PM_XZ_THREADS=1 forces one block (what the reference writes);
// PM_XZ_BLOCK sets the block size; the thread count only sets how many blocks are encoded at
// once.
constexpr uint64_t kXzBlock = (uint64_t)1 << 20;
constexpr uint64_t kXzMinBlock = (uint64_t)1 << 16;

uint64_t xz_block_size(size_t n) {
    uint64_t b = kXzMinBlock;
    while (b < kXzBlock && b * 16 < n) b <<= 1;
    return b;
}

bool xz_encode(const uint8_t* in, size_t n, std::vector<uint8_t>& out, std::string& err) {
    pm_lzma_stream s{};
    bool one_block = false;
    if (const char* e = std::getenv("PM_XZ_THREADS")) one_block |= std::atoi(e) <= 1;
    uint64_t block = xz_block_size(n);
    if (const char* e = std::getenv("PM_XZ_BLOCK")) block = std::max<uint64_t>(4096, std::strtoull(e, nullptr, 10));
    if ((n + block - 1) / block <= 1) one_block = true;
    const int threads = one_block ? 1 : (int)std::max<uint64_t>(2, std::min<uint64_t>((uint64_t)host_threads(), (n + block - 1) / block));
    const uint64_t reach = one_block ? std::max<uint64_t>(n, 1) : block;
    uint32_t dict = 4096;
    while (dict < reach && dict < ((uint32_t)64 << 20)) dict <<= 1;
    alignas(16) unsigned char opt[512] = {0};   // lzma_options_lzma (opaque past dict_size)
    if (lzma_lzma_preset(opt, 9)) { err = "xz preset"; return false; }
    uint32_t* dict_size = reinterpret_cast<uint32_t*>(opt);
    *dict_size = std::min(*dict_size, dict);
    const pm_lzma_filter filters[2] = {{0x21 /* LZMA2 */, opt}, {UINT64_MAX, nullptr}};
    if (!one_block) {
        pm_lzma_mt mt{};
        mt.threads = (uint32_t)threads;
        mt.block_size = block;
        mt.preset = 9;
        mt.filters = filters;
        mt.check = kLzmaCheckCrc64;
        if (lzma_stream_encoder_mt(&s, &mt) != kLzmaOk) { err = "xz encoder init"; return false; }
    } else if (lzma_stream_encoder(&s, filters, kLzmaCheckCrc64) != kLzmaOk) {
        err = "xz encoder init";
        return false;
    }
    out.resize(n / 2 + (1 << 16));
    s.next_in = in;
    s.avail_in = n;
    size_t done = 0;
    for (;;) {
        s.next_out = out.data() + done;
        s.avail_out = out.size() - done;
        const int rc = lzma_code(&s, kLzmaFinish);
        done = out.size() - s.avail_out;
        if (rc == kLzmaStreamEnd) break;
        if (rc != kLzmaOk) { lzma_end(&s); err = "xz encode error"; return false; }
        if (s.avail_out == 0) out.resize(out.size() * 2);
    }
    lzma_end(&s);
    out.resize(done);
    return true;
}

// ---- Cap'n Proto reader ---------------------------------------------------------------
struct Msg {
    Bytes bytes;
    std::vector<const uint64_t*> seg;
    std::vector<size_t> len;
    std::string err;

    bool init() {
        if (bytes.size() < 8) return fail("message too short");
        const uint32_t* h = reinterpret_cast<const uint32_t*>(bytes.data());
        const size_t count = (size_t)h[0] + 1;
        const size_t header = ((count + 1) * 4 + 7) / 8 * 8;
        if (count > (1u << 20) || header > bytes.size()) return fail("bad segment table");
        size_t at = header;
        for (size_t i = 0; i < count; ++i) {
            const size_t w = h[1 + i];
            if (at + w * 8 > bytes.size()) return fail("segment beyond the message");
            seg.push_back(reinterpret_cast<const uint64_t*>(bytes.data() + at));
            len.push_back(w);
            at += w * 8;
        }
        return true;
    }
    bool fail(const std::string& m) {
        if (err.empty()) err = m;
        return false;
    }
};

struct Ref {   // where an object's content starts, after resolving far pointers
    int32_t seg = -1;
    size_t pos = 0;
    uint64_t tag = 0;   // the pointer word describing the layout (offset field ignored)
};

struct Struct {
    const Msg* m = nullptr;
    int32_t seg = -1;
    size_t data = 0;
    uint16_t dwords = 0, ptrs = 0;

    uint64_t word(int i) const { return i < dwords ? m->seg[seg][data + i] : 0; }
    uint32_t u32(int bit) const { return (uint32_t)(word(bit / 64) >> (bit % 64)); }
    int32_t i32(int bit) const { return (int32_t)u32(bit); }
    int64_t i64(int bit) const { return (int64_t)word(bit / 64); }
    bool flag(int bit) const { return (word(bit / 64) >> (bit % 64)) & 1u; }
    bool has_ptr(int i) const { return i < ptrs; }
    size_t ptr_pos(int i) const { return data + dwords + i; }
};

struct List {
    const Msg* m = nullptr;
    int32_t seg = -1;
    size_t pos = 0;
    int esize = 0;
    uint32_t count = 0;
    uint16_t dwords = 0, ptrs = 0;   // composite element layout

    Struct at(uint32_t i) const {
        Struct s;
        s.m = m;
        s.seg = seg;
        s.data = pos + (size_t)i * (dwords + ptrs);
        s.dwords = dwords;
        s.ptrs = ptrs;
        return s;
    }
    uint64_t raw(uint32_t i) const {   // primitive element i (bits / bytes / words)
        const uint8_t* base = reinterpret_cast<const uint8_t*>(m->seg[seg] + pos);
        switch (esize) {
            case 1: return (base[i / 8] >> (i % 8)) & 1u;
            case 2: return base[i];
            case 3: return reinterpret_cast<const uint16_t*>(base)[i];
            case 4: return reinterpret_cast<const uint32_t*>(base)[i];
            case 5: return reinterpret_cast<const uint64_t*>(base)[i];
            default: return 0;
        }
    }
};

bool resolve(Msg& m, int32_t seg, size_t pos, Ref& out, bool& null) {
    if (seg < 0 || (size_t)seg >= m.seg.size() || pos >= m.len[seg]) return m.fail("pointer outside its segment");
    uint64_t w = m.seg[seg][pos];
    null = w == 0;
    if (null) return true;
    const int kind = (int)(w & 3);
    if (kind == 2) {   // far pointer
        const bool dbl = (w >> 2) & 1;
        const size_t pad = (size_t)((w >> 3) & 0x1FFFFFFF);
        const uint32_t ps = (uint32_t)(w >> 32);
        if (ps >= m.seg.size() || pad + (dbl ? 2 : 1) > m.len[ps]) return m.fail("bad far pointer");
        if (!dbl) return resolve(m, (int32_t)ps, pad, out, null);
        const uint64_t land = m.seg[ps][pad];
        const uint64_t tag = m.seg[ps][pad + 1];
        if ((land & 7) != 2) return m.fail("bad double-far landing pad");
        const uint32_t ts = (uint32_t)(land >> 32);
        const size_t tpos = (size_t)((land >> 3) & 0x1FFFFFFF);
        if (ts >= m.seg.size() || tpos > m.len[ts]) return m.fail("bad double-far target");
        out = Ref{(int32_t)ts, tpos, tag};
        return true;
    }
    if (kind == 3) return m.fail("capability pointer in a PanMAN");
    const int32_t off = (int32_t)(uint32_t)w >> 2;   // signed 30-bit word offset
    const int64_t target = (int64_t)pos + 1 + off;
    if (target < 0 || (size_t)target > m.len[seg]) return m.fail("pointer offset out of range");
    out = Ref{seg, (size_t)target, w};
    return true;
}

bool read_struct(Msg& m, int32_t seg, size_t pos, Struct& s) {
    Ref r;
    bool null = false;
    if (!resolve(m, seg, pos, r, null)) return false;
    s = Struct{};
    s.m = &m;
    if (null) return true;
    if ((r.tag & 3) != 0) return m.fail("expected a struct pointer");
    s.seg = r.seg;
    s.data = r.pos;
    s.dwords = (uint16_t)(r.tag >> 32);
    s.ptrs = (uint16_t)(r.tag >> 48);
    if (s.data + s.dwords + s.ptrs > m.len[s.seg]) return m.fail("struct beyond its segment");
    return true;
}

bool read_list(Msg& m, int32_t seg, size_t pos, List& l) {
    Ref r;
    bool null = false;
    if (!resolve(m, seg, pos, r, null)) return false;
    l = List{};
    l.m = &m;
    if (null) return true;
    if ((r.tag & 3) != 1) return m.fail("expected a list pointer");
    l.seg = r.seg;
    l.esize = (int)((r.tag >> 32) & 7);
    const uint32_t n = (uint32_t)(r.tag >> 35);
    if (l.esize == 7) {
        if (r.pos >= m.len[r.seg]) return m.fail("composite tag outside the segment");
        const uint64_t tag = m.seg[r.seg][r.pos];
        l.count = (uint32_t)((uint32_t)tag >> 2);
        l.dwords = (uint16_t)(tag >> 32);
        l.ptrs = (uint16_t)(tag >> 48);
        l.pos = r.pos + 1;
        if ((uint64_t)l.count * (l.dwords + l.ptrs) > n || l.pos + n > m.len[r.seg]) return m.fail("bad composite list");
    } else {
        l.count = n;
        l.pos = r.pos;
        static const int bits[7] = {0, 1, 8, 16, 32, 64, 64};
        const uint64_t words = ((uint64_t)n * bits[l.esize] + 63) / 64;
        if (l.pos + words > m.len[r.seg]) return m.fail("list beyond its segment");
        if (l.esize == 6) { l.dwords = 0; l.ptrs = 1; }
    }
    return true;
}

bool read_text(Msg& m, const Struct& s, int ptr, std::string& out) {
    out.clear();
    if (!s.has_ptr(ptr)) return true;
    List l;
    if (!read_list(m, s.seg, s.ptr_pos(ptr), l)) return false;
    if (l.seg < 0) return true;
    if (l.esize != 2) return m.fail("text is not a byte list");
    const char* p = reinterpret_cast<const char*>(m.seg[l.seg] + l.pos);
    out.assign(p, l.count > 0 ? l.count - 1 : 0);   // drop the NUL terminator
    return true;
}

bool child_list(Msg& m, const Struct& s, int ptr, List& l) {
    l = List{};
    l.m = &m;
    if (!s.has_ptr(ptr) || s.seg < 0) return true;
    return read_list(m, s.seg, s.ptr_pos(ptr), l);
}

}  // namespace

namespace {

bool load_tree(Msg& m, const Struct& t, PanmanTree& out) {
    // Newick -> nodes in pre-order (== the order of the stored node list)
    if (!read_text(m, t, 0, out.newick)) return false;
    Topology topo;
    std::string err;
    if (!parse_topology(out.newick, topo, err)) return m.fail("newick: " + err);
    const int32_t N = (int32_t)topo.name.size();
    out.num_nodes = N;
    out.root = topo.root;
    out.length = topo.length;
    out.child_off.assign(N + 1, 0);
    for (int32_t i = 0; i < N; ++i) {
        out.child_idx.insert(out.child_idx.end(), topo.kids[i].begin(), topo.kids[i].end());
        out.child_off[i + 1] = (int32_t)out.child_idx.size();
    }
    std::unordered_map<std::string, int32_t> index;
    for (int32_t i = 0; i < N; ++i) {
        out.names_blob += topo.name[i];
        out.names_blob.push_back('\0');
        index[topo.name[i]] = i;
    }
    // nodes: assignMutationsToNodes walks the tree in pre-order (src/panman.cpp:576-618).  Two
    // passes over node ranges on host threads: each node's mutation counts, then -- at offsets
    // from their prefix sums -- the flattened mutations (the message is only read: no state)
    List nodes;
    if (!child_list(m, t, 1, nodes)) return false;
    out.bm_off.assign(N + 1, 0);
    out.nm_off.assign(N + 1, 0);
    const int32_t NV = std::min<int32_t>(N, (int32_t)std::min<uint32_t>(nodes.count, (uint32_t)INT32_MAX));
    const int32_t chunk = 4096, tasks = (NV + chunk - 1) / chunk;
    std::atomic<bool> bad{false};
    host_parallel_for(tasks, [&](int task) {
        for (int32_t v = task * chunk; v < std::min(NV, (task + 1) * chunk) && !bad; ++v) {
            const Struct node = nodes.at((uint32_t)v);
            List muts;
            if (!child_list(m, node, 0, muts)) { bad = true; return; }
            int64_t nn = 0, nb = 0;
            for (uint32_t k = 0; k < muts.count; ++k) {
                const Struct mu = muts.at(k);
                List nucs;
                if (!child_list(m, mu, 0, nucs)) { bad = true; return; }
                nn += nucs.count;
                nb += mu.flag(65) ? 1 : 0;
            }
            out.nm_off[v + 1] = nn;
            out.bm_off[v + 1] = nb;
        }
    });
    if (bad) return false;
    for (int32_t v = 0; v < N; ++v) {
        out.nm_off[v + 1] += out.nm_off[v];
        out.bm_off[v + 1] += out.bm_off[v];
    }
    const size_t NM = (size_t)out.nm_off[N], BM = (size_t)out.bm_off[N];
    out.nm_primary.resize(NM);
    out.nm_secondary.resize(NM);
    out.nm_pos.resize(NM);
    out.nm_gap.resize(NM);
    out.nm_info.resize(NM);
    out.nm_nucs.resize(NM);
    out.bm_primary.resize(BM);
    out.bm_info.resize(BM);
    out.bm_inv.resize(BM);
    host_parallel_for(tasks, [&](int task) {
        for (int32_t v = task * chunk; v < std::min(NV, (task + 1) * chunk); ++v) {
            const Struct node = nodes.at((uint32_t)v);
            List muts;
            (void)child_list(m, node, 0, muts);
            size_t a = (size_t)out.nm_off[v], bi = (size_t)out.bm_off[v];
            for (uint32_t k = 0; k < muts.count; ++k) {
                const Struct mu = muts.at(k);
                const int64_t block_id = mu.i64(0);
                const bool gap_exist = mu.flag(64);
                const int32_t primary = (int32_t)(block_id >> 32);
                const int32_t secondary = gap_exist ? (int32_t)(block_id & 0xFFFFFFFF) : -1;
                List nucs;
                (void)child_list(m, mu, 0, nucs);
                for (uint32_t j = 0; j < nucs.count; ++j, ++a) {
                    const Struct nm = nucs.at(j);
                    const uint32_t info = nm.u32(96);
                    const uint32_t len = (info & 0xFF) >> 4;
                    out.nm_primary[a] = primary;
                    out.nm_secondary[a] = secondary;
                    out.nm_pos[a] = nm.i32(0);
                    out.nm_gap[a] = nm.flag(64) ? nm.i32(32) : -1;
                    out.nm_info[a] = (uint8_t)(info & 0xFF);
                    out.nm_nucs[a] = len <= 6 ? (info >> 8) << (24 - 4 * len) : 0;
                }
                if (mu.flag(65)) {   // blockMutExist
                    out.bm_primary[bi] = primary;
                    out.bm_info[bi] = mu.flag(66);
                    out.bm_inv[bi] = mu.flag(67);
                    ++bi;
                }
            }
        }
    });
    // blocks in (primary, secondary) order (std::map, src/panman.cpp:1668-1724)
    std::map<std::pair<int32_t, int32_t>, std::vector<uint32_t>> blocks;
    List cmap;
    if (!child_list(m, t, 2, cmap)) return false;
    for (uint32_t k = 0; k < cmap.count; ++k) {
        const Struct c = cmap.at(k);
        List ids, seq, gapx;
        if (!child_list(m, c, 0, ids) || !child_list(m, c, 1, seq) || !child_list(m, c, 2, gapx)) return false;
        std::vector<uint32_t> words(seq.count);
        for (uint32_t j = 0; j < seq.count; ++j) words[j] = (uint32_t)seq.raw(j);
        for (uint32_t j = 0; j < ids.count; ++j) {
            const int64_t id = (int64_t)ids.raw(j);
            const bool gx = j < gapx.count && gapx.raw(j);
            blocks[{(int32_t)(id >> 32), gx ? (int32_t)(id & 0xFFFFFFFF) : -1}] = words;
        }
    }
    out.block_seq_off.push_back(0);
    for (auto& b : blocks) {
        out.block_primary.push_back(b.first.first);
        out.block_seq.insert(out.block_seq.end(), b.second.begin(), b.second.end());
        out.block_seq_off.push_back((int64_t)out.block_seq.size());
    }
    // gaps
    List gaps;
    if (!child_list(m, t, 3, gaps)) return false;
    out.gap_off.push_back(0);
    for (uint32_t k = 0; k < gaps.count; ++k) {
        const Struct g = gaps.at(k);
        List len, pos;
        if (!child_list(m, g, 0, len) || !child_list(m, g, 1, pos)) return false;
        out.gap_primary.push_back((int32_t)(g.i64(0) >> 32));
        for (uint32_t j = 0; j < pos.count; ++j) {
            out.gap_pos.push_back((uint32_t)pos.raw(j));
            out.gap_len.push_back(j < len.count ? (uint32_t)len.raw(j) : 0);
        }
        out.gap_off.push_back((int64_t)out.gap_pos.size());
    }
    // circular offsets, rotation indexes, inversions (by sequence id)
    out.circular.assign(N, -1);
    out.rotation.assign(N, 0);
    out.inverted.assign(N, 0);
    for (int ptr = 5; ptr <= 7; ++ptr) {
        List l;
        if (!child_list(m, t, ptr, l)) return false;
        for (uint32_t k = 0; k < l.count; ++k) {
            const Struct e = l.at(k);
            std::string id;
            if (!read_text(m, e, 0, id)) return false;
            auto it = index.find(id);
            if (it == index.end()) continue;
            if (ptr == 5) out.circular[it->second] = e.i32(0);
            else if (ptr == 6) out.rotation[it->second] = e.i32(0);
            else out.inverted[it->second] = e.flag(0);
        }
    }
    return true;
}

// ---- Protobuf (panmanOld, panman.proto) ------------------------------------------------
struct Pb {
    const uint8_t* p;
    const uint8_t* end;
    std::string* err;
    bool fail(const char* what) {
        if (err && err->empty()) *err = std::string("protobuf: ") + what;
        return false;
    }
    bool varint(uint64_t& v) {
        v = 0;
        for (int sh = 0; sh < 64; sh += 7) {
            if (p >= end) return fail("truncated varint");
            const uint8_t b = *p++;
            v |= (uint64_t)(b & 0x7F) << sh;
            if (!(b & 0x80)) return true;
        }
        return fail("varint too long");
    }
    // next field: number, wire type; length-delimited payloads in [sub, sub_end)
    bool next(uint32_t& field, uint32_t& wire, uint64_t& value, const uint8_t*& sub, const uint8_t*& sub_end) {
        uint64_t key;
        if (!varint(key)) return false;
        field = (uint32_t)(key >> 3);
        wire = (uint32_t)(key & 7);
        if (field == 0) return fail("field number 0");
        switch (wire) {
            case 0: return varint(value);
            case 1:
                if (end - p < 8) return fail("truncated fixed64");
                std::memcpy(&value, p, 8);
                p += 8;
                return true;
            case 5: {
                if (end - p < 4) return fail("truncated fixed32");
                uint32_t v32;
                std::memcpy(&v32, p, 4);
                value = v32;
                p += 4;
                return true;
            }
            case 2: {
                uint64_t n;
                if (!varint(n)) return false;
                if (n > (uint64_t)(end - p)) return fail("length past the end");
                sub = p;
                sub_end = p + n;
                p += n;
                return true;
            }
            default: return fail("unsupported wire type (groups)");
        }
    }
};

// A repeated varint field, packed (wire 2) or not (wire 0): append its value(s).
template <class T>
bool pb_repeated(Pb& r, uint32_t wire, uint64_t value, const uint8_t* sub, const uint8_t* sub_end, std::vector<T>& out) {
    if (wire == 0) {
        out.push_back((T)value);
        return true;
    }
    if (wire != 2) return r.fail("repeated scalar with a bad wire type");
    Pb q{sub, sub_end, r.err};
    while (q.p < q.end) {
        uint64_t v;
        if (!q.varint(v)) return false;
        out.push_back((T)v);
    }
    return true;
}

// Walk a message's fields, calling f(field, wire, value, sub, sub_end) for each.
template <class F>
bool pb_fields(const uint8_t* b, const uint8_t* e, std::string& err, F&& f) {
    Pb r{b, e, &err};
    while (r.p < r.end) {
        uint32_t field, wire;
        uint64_t value = 0;
        const uint8_t *sub = nullptr, *sub_end = nullptr;
        if (!r.next(field, wire, value, sub, sub_end)) return false;
        if (!f(r, field, wire, value, sub, sub_end)) return false;
    }
    return true;
}

struct PbNucMut {
    int32_t pos = 0, gap_pos = 0;
    bool gap_exist = false;
    uint32_t info = 0;
};
struct PbMutation {
    int64_t block_id = 0;
    bool gap_exist = false, mut_exist = false, mut_info = false, inversion = false;
    std::vector<PbNucMut> nucs;
};

bool pb_mutation(const uint8_t* b, const uint8_t* e, std::string& err, PbMutation& mu) {
    return pb_fields(b, e, err, [&](Pb& r, uint32_t f, uint32_t w, uint64_t v, const uint8_t* sb, const uint8_t* se) {
        switch (f) {
            case 1: mu.block_id = (int64_t)v; return true;
            case 2: mu.gap_exist = v != 0; return true;
            case 3: mu.mut_exist = v != 0; return true;
            case 4: mu.mut_info = v != 0; return true;
            case 5: mu.inversion = v != 0; return true;
            case 6: {
                if (w != 2) return r.fail("nucMutation is not a message");
                PbNucMut nm;
                const bool ok = pb_fields(sb, se, err, [&](Pb&, uint32_t g, uint32_t, uint64_t x, const uint8_t*, const uint8_t*) {
                    if (g == 1) nm.pos = (int32_t)x;           // int32: 64-bit two's complement varint
                    else if (g == 2) nm.gap_pos = (int32_t)x;
                    else if (g == 3) nm.gap_exist = x != 0;
                    else if (g == 4) nm.info = (uint32_t)x;
                    return true;
                });
                if (ok) mu.nucs.push_back(nm);
                return ok;
            }
            default: return true;   // unknown fields are skipped, as protobuf does
        }
    });
}

bool load_tree_pb(const uint8_t* b, const uint8_t* e, PanmanTree& out, std::string& err) {
    // the tree's fields, gathered first (protobuf field order is free)
    std::vector<std::pair<const uint8_t*, const uint8_t*>> nodes, cmaps, gaps, named[3];
    bool have_newick = false;
    const bool ok = pb_fields(b, e, err, [&](Pb& r, uint32_t f, uint32_t w, uint64_t, const uint8_t* sb, const uint8_t* se) {
        if (f == 1 || f == 2 || (f >= 4 && f <= 9)) {
            if (w != 2) return r.fail("tree field is not length-delimited");
        }
        switch (f) {
            case 1: out.newick.assign((const char*)sb, (size_t)(se - sb)); have_newick = true; return true;
            case 2: nodes.emplace_back(sb, se); return true;
            case 4: cmaps.emplace_back(sb, se); return true;
            case 5: gaps.emplace_back(sb, se); return true;
            case 6: return true;   // blockGaps: never used by the drivers (see load_tree)
            case 7: named[0].emplace_back(sb, se); return true;
            case 8: named[1].emplace_back(sb, se); return true;
            case 9: named[2].emplace_back(sb, se); return true;
            default: return true;
        }
    });
    if (!ok) return false;
    if (!have_newick) { err = "protobuf: tree without a newick string"; return false; }
    Topology topo;
    if (!parse_topology(out.newick, topo, err)) { err = "newick: " + err; return false; }
    const int32_t N = (int32_t)topo.name.size();
    out.num_nodes = N;
    out.root = topo.root;
    out.length = topo.length;
    out.child_off.assign(N + 1, 0);
    for (int32_t i = 0; i < N; ++i) {
        out.child_idx.insert(out.child_idx.end(), topo.kids[i].begin(), topo.kids[i].end());
        out.child_off[i + 1] = (int32_t)out.child_idx.size();
    }
    std::unordered_map<std::string, int32_t> index;
    for (int32_t i = 0; i < N; ++i) {
        out.names_blob += topo.name[i];
        out.names_blob.push_back('\0');
        index[topo.name[i]] = i;
    }
    // nodes: i-th stored node = i-th node in pre-order (assignMutationsToNodes)
    out.bm_off.assign(N + 1, 0);
    out.nm_off.assign(N + 1, 0);
    for (int32_t v = 0; v < N; ++v) {
        if ((size_t)v < nodes.size()) {
            std::vector<PbMutation> muts;
            if (!pb_fields(nodes[v].first, nodes[v].second, err,
                           [&](Pb& r, uint32_t f, uint32_t w, uint64_t, const uint8_t* sb, const uint8_t* se) {
                               if (f != 1) return true;   // annotations (2) are not on this path
                               if (w != 2) return r.fail("mutation is not a message");
                               muts.emplace_back();
                               return pb_mutation(sb, se, err, muts.back());
                           }))
                return false;
            // NucMuts of every mutation first, then the block mutations (src/panman.cpp:1775-1790)
            for (const PbMutation& mu : muts) {
                const int32_t primary = (int32_t)(mu.block_id >> 32);
                const int32_t secondary = mu.gap_exist ? (int32_t)(mu.block_id & 0xFFFFFFFF) : -1;
                for (const PbNucMut& nm : mu.nucs) {
                    const uint32_t info = nm.info & 0xFF, len = info >> 4;
                    out.nm_primary.push_back(primary);
                    out.nm_secondary.push_back(secondary);
                    out.nm_pos.push_back(nm.pos);
                    out.nm_gap.push_back(nm.gap_exist ? nm.gap_pos : -1);
                    out.nm_info.push_back((uint8_t)info);
                    out.nm_nucs.push_back(len <= 6 ? (nm.info >> 8) << (24 - 4 * len) : 0);
                }
            }
            for (const PbMutation& mu : muts)
                if (mu.mut_exist) {
                    out.bm_primary.push_back((int32_t)(mu.block_id >> 32));
                    out.bm_info.push_back(mu.mut_info);
                    out.bm_inv.push_back(mu.inversion);
                }
        }
        out.bm_off[v + 1] = (int64_t)out.bm_primary.size();
        out.nm_off[v + 1] = (int64_t)out.nm_primary.size();
    }
    // blocks in (primary, secondary) order (std::map, src/panman.cpp:1806-1822, :1829-1832)
    std::map<std::pair<int32_t, int32_t>, std::vector<uint32_t>> blocks;
    for (const auto& c : cmaps) {
        std::vector<int64_t> ids;
        std::vector<uint32_t> seq;
        std::vector<uint8_t> gapx;
        if (!pb_fields(c.first, c.second, err, [&](Pb& r, uint32_t f, uint32_t w, uint64_t v, const uint8_t* sb, const uint8_t* se) {
                if (f == 1) return pb_repeated(r, w, v, sb, se, ids);
                if (f == 2) return pb_repeated(r, w, v, sb, se, seq);
                if (f == 3) return pb_repeated(r, w, v, sb, se, gapx);
                return true;   // chromosomeName (4)
            }))
            return false;
        for (size_t j = 0; j < ids.size(); ++j) {
            const bool gx = j < gapx.size() && gapx[j];
            blocks[{(int32_t)(ids[j] >> 32), gx ? (int32_t)(ids[j] & 0xFFFFFFFF) : -1}] = seq;
        }
    }
    out.block_seq_off.push_back(0);
    for (auto& bk : blocks) {
        out.block_primary.push_back(bk.first.first);
        out.block_seq.insert(out.block_seq.end(), bk.second.begin(), bk.second.end());
        out.block_seq_off.push_back((int64_t)out.block_seq.size());
    }
    // gaps (src/panman.cpp:1835-1845)
    out.gap_off.push_back(0);
    for (const auto& g : gaps) {
        int64_t block_id = 0;
        std::vector<int32_t> len, pos;
        if (!pb_fields(g.first, g.second, err, [&](Pb& r, uint32_t f, uint32_t w, uint64_t v, const uint8_t* sb, const uint8_t* se) {
                if (f == 1) block_id = (int64_t)v;
                else if (f == 3) return pb_repeated(r, w, v, sb, se, len);
                else if (f == 4) return pb_repeated(r, w, v, sb, se, pos);
                return true;
            }))
            return false;
        out.gap_primary.push_back((int32_t)(block_id >> 32));
        for (size_t j = 0; j < pos.size(); ++j) {
            out.gap_pos.push_back((uint32_t)pos[j]);
            out.gap_len.push_back(j < len.size() ? (uint32_t)len[j] : 0);
        }
        out.gap_off.push_back((int64_t)out.gap_pos.size());
    }
    // circular offsets, rotation indexes, inversions by sequence id (:1847-1860)
    out.circular.assign(N, -1);
    out.rotation.assign(N, 0);
    out.inverted.assign(N, 0);
    for (int k = 0; k < 3; ++k)
        for (const auto& x : named[k]) {
            std::string id;
            int64_t value = 0;
            if (!pb_fields(x.first, x.second, err, [&](Pb&, uint32_t f, uint32_t, uint64_t v, const uint8_t* sb, const uint8_t* se) {
                    if (f == 1) id.assign((const char*)sb, (size_t)(se - sb));
                    else if (f == 2) value = (int64_t)v;
                    return true;
                }))
                return false;
            auto it = index.find(id);
            if (it == index.end()) continue;
            if (k == 0) out.circular[it->second] = (int32_t)value;
            else if (k == 1) out.rotation[it->second] = (int32_t)value;
            else out.inverted[it->second] = value != 0;
        }
    return true;
}

// ---- Cap'n Proto writer (one segment) ---------------------------------------------------
struct Writer {
    std::vector<uint64_t> w{0};   // word 0: root pointer

    size_t alloc(size_t words) {
        const size_t at = w.size();
        w.resize(at + words, 0);
        return at;
    }
    void struct_ptr(size_t ptr, size_t target, uint16_t dwords, uint16_t ptrs) {
        const int64_t off = (int64_t)target - (int64_t)(ptr + 1);
        w[ptr] = ((uint64_t)(uint32_t)(off << 2)) | ((uint64_t)dwords << 32) | ((uint64_t)ptrs << 48);
    }
    void list_ptr(size_t ptr, size_t target, int esize, uint64_t count) {
        const int64_t off = (int64_t)target - (int64_t)(ptr + 1);
        w[ptr] = ((uint64_t)(uint32_t)(off << 2)) | 1u | ((uint64_t)esize << 32) | (count << 35);
    }
    // composite list of n structs; returns the position of element 0
    size_t composite(size_t ptr, uint32_t n, uint16_t dwords, uint16_t ptrs) {
        const size_t per = (size_t)dwords + ptrs;
        const size_t tag = alloc(1 + per * n);
        list_ptr(ptr, tag, 7, per * n);
        w[tag] = ((uint64_t)n << 2) | ((uint64_t)dwords << 32) | ((uint64_t)ptrs << 48);
        return tag + 1;
    }
    template <class T>
    void prim_list(size_t ptr, const std::vector<T>& v, int esize) {
        static const int bits[7] = {0, 1, 8, 16, 32, 64, 64};
        const size_t words = (v.size() * bits[esize] + 63) / 64;
        const size_t at = alloc(words);
        uint8_t* base = reinterpret_cast<uint8_t*>(w.data() + at);
        for (size_t i = 0; i < v.size(); ++i) {
            if (esize == 1) base[i / 8] |= (uint8_t)((v[i] ? 1 : 0) << (i % 8));
            else std::memcpy(base + i * (bits[esize] / 8), &v[i], bits[esize] / 8);
        }
        list_ptr(ptr, at, esize, v.size());
    }
    void text(size_t ptr, const std::string& s) {
        const size_t at = alloc((s.size() + 1 + 7) / 8);
        std::memcpy(w.data() + at, s.data(), s.size());
        list_ptr(ptr, at, 2, s.size() + 1);
    }
    void set_u32(size_t word, int bit, uint32_t v) { w[word + bit / 64] |= (uint64_t)v << (bit % 64); }
    void set_i64(size_t word, int64_t v) { w[word] = (uint64_t)v; }
    void set_bit(size_t word, int bit, bool v) {
        if (v) w[word + bit / 64] |= 1ull << (bit % 64);
    }
};

void write_tree(Writer& wr, size_t tree_pos, const pm_panmat& p) {
    const int32_t N = p.num_nodes;
    std::vector<std::string> names(N);
    const char* nm = p.names;
    for (int32_t i = 0; i < N; ++i) {
        names[i] = nm;
        nm += names[i].size() + 1;
    }
    Topology topo;
    topo.name = names;
    topo.kids.assign(N, {});
    topo.root = p.root;
    if (p.branch_length) topo.length.assign(p.branch_length, p.branch_length + N);
    for (int32_t i = 0; i < N; ++i)
        for (int32_t e = p.child_offsets[i]; e < p.child_offsets[i + 1]; ++e) topo.kids[i].push_back(p.child_index[e]);
    // ptr slots of the Tree struct are at tree_pos + k (0 data words)
    wr.text(tree_pos + 0, newick_of(topo));
    // nodes in pre-order, plus the trailing empty node the reference writes (:6898)
    std::vector<int32_t> pre;
    std::vector<int32_t> st{p.root};
    while (!st.empty()) {
        const int32_t v = st.back();
        st.pop_back();
        pre.push_back(v);
        for (int32_t e = p.child_offsets[v + 1] - 1; e >= p.child_offsets[v]; --e) st.push_back(p.child_index[e]);
    }
    const size_t nodes = wr.composite(tree_pos + 1, (uint32_t)N + 1, 0, 2);
    for (int32_t k = 0; k < N; ++k) {
        const int32_t v = pre[k];
        const size_t node = nodes + (size_t)k * 2;
        // group by (primary, secondary) in std::map order (:2857-2887)
        struct Group { std::vector<int64_t> nucs; int block = 2; bool inv = false; };
        std::map<std::pair<int32_t, int32_t>, Group> groups;
        for (int64_t i = p.nuc_mut_offsets[v]; i < p.nuc_mut_offsets[v + 1]; ++i)
            groups[{p.nuc_mut_primary[i], p.nuc_mut_secondary ? p.nuc_mut_secondary[i] : -1}].nucs.push_back(i);
        for (int64_t i = p.block_mut_offsets[v]; i < p.block_mut_offsets[v + 1]; ++i) {
            Group& g = groups[{p.block_mut_primary[i], -1}];
            g.block = p.block_mut_info[i] ? 1 : 0;
            g.inv = p.block_mut_inversion[i] != 0;
        }
        const size_t muts = wr.composite(node + 0, (uint32_t)groups.size(), 2, 1);
        size_t gi = 0;
        for (auto& kv : groups) {
            const size_t mu = muts + gi++ * 3;
            const int32_t prim = kv.first.first, sec = kv.first.second;
            wr.set_i64(mu, sec != -1 ? ((int64_t)prim << 32) + sec : ((int64_t)prim << 32));
            wr.set_bit(mu, 64, sec != -1);
            wr.set_bit(mu, 65, kv.second.block != 2);
            wr.set_bit(mu, 66, kv.second.block != 0);   // setBlockMutInfo(2) stores true (:2889)
            wr.set_bit(mu, 67, kv.second.block != 2 ? kv.second.inv : true);
            const size_t nl = wr.composite(mu + 2, (uint32_t)kv.second.nucs.size(), 2, 0);
            for (size_t j = 0; j < kv.second.nucs.size(); ++j) {
                const int64_t i = kv.second.nucs[j];
                const size_t rec = nl + j * 2;
                const uint32_t info = p.nuc_mut_info[i];
                const uint32_t len = info >> 4;
                const uint32_t disk = len <= 6 ? (((p.nuc_mut_nucs[i] >> (24 - 4 * len)) << 8) + info) : info;
                wr.set_u32(rec, 0, (uint32_t)p.nuc_mut_position[i]);
                if (p.nuc_mut_gap_position[i] != -1) {
                    wr.set_u32(rec, 32, (uint32_t)p.nuc_mut_gap_position[i]);
                    wr.set_bit(rec, 64, true);
                }
                wr.set_u32(rec, 96, disk);
            }
        }
        wr.composite(node + 1, 0, 0, 1);   // annotations: empty list of text
    }
    // consensusSeqMap: blocks grouped by identical consensus words, in map order
    std::map<std::vector<uint32_t>, std::vector<int64_t>> by_seq;
    for (int32_t b = 0; b < p.num_blocks; ++b) {
        std::vector<uint32_t> words(p.block_seq + p.block_seq_offsets[b], p.block_seq + p.block_seq_offsets[b + 1]);
        by_seq[words].push_back((int64_t)p.block_primary[b] << 32);
    }
    const size_t cm = wr.composite(tree_pos + 2, (uint32_t)by_seq.size(), 0, 4);
    size_t ci = 0;
    for (auto& kv : by_seq) {
        const size_t c = cm + ci++ * 4;
        wr.prim_list(c + 0, kv.second, 5);
        wr.prim_list(c + 1, kv.first, 4);
        wr.prim_list(c + 2, std::vector<uint8_t>(kv.second.size(), 0), 1);
        wr.composite(c + 3, 0, 0, 1);   // chromosomeName: empty
    }
    // gaps
    const size_t gl = wr.composite(tree_pos + 3, (uint32_t)p.num_gaps, 2, 2);
    for (int32_t g = 0; g < p.num_gaps; ++g) {
        const size_t e = gl + (size_t)g * 4;
        wr.set_i64(e, (int64_t)p.gap_primary[g] << 32);
        std::vector<int32_t> len, pos;
        for (int64_t k = p.gap_offsets[g]; k < p.gap_offsets[g + 1]; ++k) {
            len.push_back((int32_t)p.gap_length[k]);
            pos.push_back((int32_t)p.gap_position[k]);
        }
        wr.prim_list(e + 2, len, 4);
        wr.prim_list(e + 3, pos, 4);
    }
    // blockGaps (ptr 4) is not written by TreeGroup::writeToFile: left null
    // circular / rotation / inverted
    std::vector<int32_t> circ, rot, inv;
    for (int32_t i = 0; i < N; ++i) {
        if (p.circular_offset && p.circular_offset[i] >= 0) circ.push_back(i);
        if (p.rotation_index && p.rotation_index[i] != 0) rot.push_back(i);
        if (p.sequence_inverted && p.sequence_inverted[i]) inv.push_back(i);
    }
    const size_t co = wr.composite(tree_pos + 5, (uint32_t)circ.size(), 1, 1);
    for (size_t k = 0; k < circ.size(); ++k) {
        wr.set_u32(co + k * 2, 0, (uint32_t)p.circular_offset[circ[k]]);
        wr.text(co + k * 2 + 1, names[circ[k]]);
    }
    const size_t ro = wr.composite(tree_pos + 6, (uint32_t)rot.size(), 1, 1);
    for (size_t k = 0; k < rot.size(); ++k) {
        wr.set_u32(ro + k * 2, 0, (uint32_t)p.rotation_index[rot[k]]);
        wr.text(ro + k * 2 + 1, names[rot[k]]);
    }
    const size_t io = wr.composite(tree_pos + 7, (uint32_t)inv.size(), 1, 1);
    for (size_t k = 0; k < inv.size(); ++k) {
        wr.set_bit(io + k * 2, 0, true);
        wr.text(io + k * 2 + 1, names[inv[k]]);
    }
}

}  // namespace
}  // namespace pm

using namespace pm;

extern "C" {

int pm_panman_load(const char* path, pm_panman** out, char* err, int64_t err_len) {
    auto set_err = [&](const std::string& e) {
        if (err && err_len > 0) std::snprintf(err, (size_t)err_len, "%s", e.c_str());
    };
    if (!path || !out) return PM_ERR_ARG;
    *out = nullptr;
    PhaseClock clock;
    FILE* f = std::fopen(path, "rb");
    if (!f) { set_err(std::string("cannot open ") + path); return PM_ERR_ARG; }
    std::vector<uint8_t> raw;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) raw.insert(raw.end(), buf, buf + n);
    std::fclose(f);
    clock.lap("panman.read_file");
    Msg m;
    std::string e;
    const bool is_xz = raw.size() >= 6 && raw[0] == 0xFD && raw[1] == '7' && raw[2] == 'z' && raw[3] == 'X';
    if (is_xz) {
        if (!xz_decode(raw, m.bytes, e)) { set_err(e); return PM_ERR_ARG; }
    } else {
        m.bytes.assign(raw.begin(), raw.end());   // an uncompressed capnp message is accepted too
    }
    clock.lap("panman.xz_decode");
    if (!m.init()) { set_err(m.err); return PM_ERR_ARG; }
    Struct tg;
    if (!read_struct(m, 0, 0, tg)) { set_err(m.err); return PM_ERR_ARG; }
    List trees;
    if (!child_list(m, tg, 0, trees)) { set_err(m.err); return PM_ERR_ARG; }
    auto* pm_ = new pm_panman();
    pm_->trees.resize(trees.count);
    for (uint32_t t = 0; t < trees.count; ++t)
        if (!load_tree(m, trees.at(t), pm_->trees[t])) {
            set_err(m.err);
            delete pm_;
            return PM_ERR_ARG;
        }
    clock.lap("panman.capnp_decode");
    *out = pm_;
    return PM_OK;
}

int pm_panman_load_old(const char* path, pm_panman** out, char* err, int64_t err_len) {
    auto set_err = [&](const std::string& e) {
        if (err && err_len > 0) std::snprintf(err, (size_t)err_len, "%s", e.c_str());
    };
    if (!path || !out) return PM_ERR_ARG;
    *out = nullptr;
    FILE* f = std::fopen(path, "rb");
    if (!f) { set_err(std::string("cannot open ") + path); return PM_ERR_ARG; }
    std::vector<uint8_t> raw;
    Bytes bytes;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) raw.insert(raw.end(), buf, buf + n);
    std::fclose(f);
    std::string e;
    const bool is_xz = raw.size() >= 6 && raw[0] == 0xFD && raw[1] == '7' && raw[2] == 'z' && raw[3] == 'X';
    if (is_xz) {
        if (!xz_decode(raw, bytes, e)) { set_err(e); return PM_ERR_ARG; }
    } else {
        bytes.assign(raw.begin(), raw.end());   // an uncompressed message is accepted too
    }
    // treeGroup: trees (1), complexMutations (2: not on this path, as in pm_panman_load)
    std::vector<std::pair<const uint8_t*, const uint8_t*>> trees;
    const uint8_t* b = bytes.data();
    if (!pb_fields(b, b + bytes.size(), e, [&](Pb& r, uint32_t fld, uint32_t w, uint64_t, const uint8_t* sb, const uint8_t* se) {
            if (fld != 1) return true;
            if (w != 2) return r.fail("tree is not a message");
            trees.emplace_back(sb, se);
            return true;
        })) {
        set_err(e);
        return PM_ERR_ARG;
    }
    if (trees.empty()) { set_err("protobuf: no tree in the tree group"); return PM_ERR_ARG; }
    auto* pm_ = new pm_panman();
    pm_->trees.resize(trees.size());
    for (size_t t = 0; t < trees.size(); ++t)
        if (!load_tree_pb(trees[t].first, trees[t].second, pm_->trees[t], e)) {
            set_err(e);
            delete pm_;
            return PM_ERR_ARG;
        }
    *out = pm_;
    return PM_OK;
}

int pm_panman_tree_count(const pm_panman* p) { return p ? (int)p->trees.size() : 0; }

int pm_panman_tree(const pm_panman* p, int index, pm_panmat* view) {
    if (!p || !view || index < 0 || index >= (int)p->trees.size()) return PM_ERR_ARG;
    p->trees[index].view(*view);
    return PM_OK;
}

const char* pm_panman_newick(const pm_panman* p, int index) {
    if (!p || index < 0 || index >= (int)p->trees.size()) return nullptr;
    return p->trees[index].newick.c_str();
}

void pm_panman_free(pm_panman* p) { delete p; }

int pm_panman_write(const char* path, const pm_panmat* const* trees, int count, int compress) {
    if (!path || (!trees && count > 0) || count < 0) return PM_ERR_ARG;
    PhaseClock clock;
    Writer wr;
    const size_t tg = wr.alloc(2);
    wr.struct_ptr(0, tg, 0, 2);
    const size_t tl = wr.composite(tg + 0, (uint32_t)count, 0, 8);
    for (int t = 0; t < count; ++t) write_tree(wr, tl + (size_t)t * 8, *trees[t]);
    wr.composite(tg + 1, 0, 10, 3);   // complexMutations: none
    std::vector<uint8_t> msg(8 + wr.w.size() * 8);
    const uint32_t hdr[2] = {0, (uint32_t)wr.w.size()};
    std::memcpy(msg.data(), hdr, 8);
    std::memcpy(msg.data() + 8, wr.w.data(), wr.w.size() * 8);
    std::vector<uint8_t> outb;
    std::string e;
    clock.lap("panman.capnp_encode");
    if (compress) {
        if (!xz_encode(msg.data(), msg.size(), outb, e)) return PM_ERR_HIP;
        clock.lap("panman.xz_encode");
    } else {
        outb.swap(msg);
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) return PM_ERR_ARG;
    const bool ok = std::fwrite(outb.data(), 1, outb.size(), f) == outb.size();
    std::fclose(f);
    clock.lap("panman.write_file");
    return ok ? PM_OK : PM_ERR_ARG;
}

}  // extern "C"
