// quadnodes.hpp -- two-level kd node records for the secondary closest and shadow traces.
//
// The kd descent (kdtree.cpp:248-281 / 322-344) makes one decision per inner node.  With the fat
// records (cr_upload_scene: a node's own 8-B word and both children's, 32 B per node) a lane loads
// two descent levels per dependent fetch, but as TWO vector-memory instructions (dwordx4 + dwordx2),
// and the traces are bound by their vector loads (the address path 0.83 busy).  A
// quad record holds the same two levels in 16 B -- ONE dwordx4:
//
//   {w_n, w_c0, w_c1, meta}   meta = axis_n | axis_c0 << 2 | axis_c1 << 4 | base << 6
//
// for a "record root" n (the tree's root and every node two levels below a record root) and its
// children c0, c1 ("middle" nodes).  An inner node's word is its split (float bits); a leaf's word is
// first | count << fbits (the scene's reference count fixes fbits) and its axis is 3.  The children of
// an inner middle node c_k are record roots at consecutive slots gb_k, gb_k + 1 with
// gb_0 = base, gb_1 = base + (c0 inner ? 2 : 0): a record root's grandchildren take one block of
// slots, allocated depth-first, so a subtree's records stay together.  A traversal position is a code
// slot << 2 | sel: sel 0 the record root, 1 / 2 its middle child c0 / c1 (a far middle child is
// pushed that way and resumes with one step of its parent's record).  Only the addresses change: a
// lane makes the same decisions at the same nodes with the same intervals (tests/native/quad_check.cpp
// models both traversals against the recursion).
//
// Host-side builder only (plain C++): cabi.cpp (cr_upload_scene) and the CPU model include it.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace cr {

// node words in cabi.cpp's encoding: x = split bits | first ref, y = axis | child << 2 (leaf: 3 | count << 2)
struct QuadNode {
    uint32_t x, y;
};

struct QuadLayout {
    std::vector<uint32_t> rec; // 4 words per slot
    uint32_t fbits = 0;        // leaf word = first | count << fbits
    uint32_t slots = 0;
};

// the leaf word of a leaf node (first, count); fbits bits of first
inline uint32_t quad_leaf_word(uint32_t first, uint32_t count, uint32_t fbits) { return first | (count << fbits); }

// Builds the records of the tree nodes[0..nn) (root 0) over nrefs references.  False (err set) when a
// leaf's first or count does not fit its word, or the slots exceed the meta word's 26 bits: the scene
// then keeps the fat-record builds.
inline bool quad_build(const QuadNode *nodes, uint32_t nn, uint32_t nrefs, QuadLayout &out, std::string &err) {
    out.rec.clear();
    out.fbits = 1;
    while (out.fbits < 31 && (1ull << out.fbits) <= (uint64_t)nrefs) out.fbits++;
    const uint32_t cmax = out.fbits >= 32 ? 0u : (uint32_t)((1ull << (32 - out.fbits)) - 1);
    auto leafy = [&](uint32_t i) { return (nodes[i].y & 3u) == 3u; };
    auto word = [&](uint32_t i, bool &ok) -> uint32_t {
        if (!leafy(i)) return nodes[i].x;
        const uint32_t first = nodes[i].x, count = nodes[i].y >> 2;
        // (count < cmax: no leaf word has all its count bits set, so 0xfffffffe -- the traces' pending
        // marker -- and 0xffffffff are never leaf words)
        if (count >= cmax || (count && (uint64_t)first >= (1ull << out.fbits))) ok = false;
        return quad_leaf_word(count ? first : 0u, count, out.fbits);
    };
    // explicit work list: (slot, node) pairs, the grandchildren block allocated when a record is written
    std::vector<std::pair<uint32_t, uint32_t>> work;
    out.rec.assign(4, 0u);
    work.emplace_back(0u, 0u);
    bool ok = true;
    while (!work.empty() && ok) {
        const auto [slot, n] = work.back();
        work.pop_back();
        uint32_t *r = out.rec.data() + 4 * (size_t)slot;
        if (leafy(n)) {
            r[0] = word(n, ok);
            r[1] = r[2] = 0u;
            r[3] = 3u;
            continue;
        }
        const uint32_t c = nodes[n].y >> 2;
        if (c + 1 >= nn) {
            err = "quad records: child out of range";
            return false;
        }
        const bool in0 = !leafy(c), in1 = !leafy(c + 1);
        const uint32_t base = (uint32_t)(out.rec.size() / 4);
        const uint32_t nb = 2u * (in0 + in1);
        if ((uint64_t)base + nb >= (1ull << 26)) {
            err = "quad records: more than 2^26 slots";
            return false;
        }
        r[0] = nodes[n].x;
        r[1] = word(c, ok);
        r[2] = word(c + 1, ok);
        r[3] = (nodes[n].y & 3u) | (nodes[c].y & 3u) << 2 | (nodes[c + 1].y & 3u) << 4 | base << 6;
        out.rec.resize(out.rec.size() + 4 * (size_t)nb, 0u); // (r is stale from here on)
        // depth-first: the first grandchild's subtree is written right after this block
        uint32_t j = base + nb;
        for (int k = 1; k >= 0; k--) {
            const uint32_t ck = c + (uint32_t)k;
            if (leafy(ck)) continue;
            const uint32_t g = nodes[ck].y >> 2;
            j -= 2;
            work.emplace_back(j + 1, g + 1);
            work.emplace_back(j, g);
        }
    }
    if (!ok) {
        err = "quad records: a leaf's first reference or count does not fit its word";
        return false;
    }
    out.slots = (uint32_t)(out.rec.size() / 4);
    return true;
}

} // namespace cr
