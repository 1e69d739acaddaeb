// Host check of the shard tile math of bh_common.hpp (compiled by tests/test_shard_math.py):
// shard_tile_coords and shard_tile_index are inverse bijections between each shard's local indices
// and the frame's tiles, agreeing with the division form shard_row_start, for S = 1..17.
#include <cstdio>
#include <initializer_list>

#include "bh_common.hpp"

int main() {
    long bad = 0, n = 0;
    for (uint32_t S = 1; S <= 17; ++S)
        for (uint32_t tiles_x : {1u, 2u, 3u, 7u, 13u, 64u, 1448u})
            for (uint32_t tiles_y : {1u, 5u, 9u, 31u, 724u}) {
                uint64_t total = 0;
                for (uint32_t k = 0; k < S; ++k) {
                    const uint64_t c = bh::shard_tile_count(tiles_x, tiles_y, k, S);
                    total += c;
                    for (uint32_t t = 0; t < c; ++t) {
                        uint32_t tx, ty, kk;
                        bh::shard_tile_coords(t, tiles_x, k, S, &tx, &ty);
                        const uint32_t tt = bh::shard_tile_index(tx, ty, tiles_x, S, &kk);
                        const uint32_t st = bh::shard_row_start(ty, k, S);
                        if (tx >= tiles_x || ty >= tiles_y || kk != k || tt != t || tx < st || (tx - st) % S) ++bad;
                        ++n;
                    }
                }
                if (total != (uint64_t)tiles_x * tiles_y) ++bad;
            }
    std::printf("checked %ld tiles, %ld bad\n", n, bad);
    return bad != 0;
}
