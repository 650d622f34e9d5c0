#pragma once
#include <cstdint>

namespace albedo {
bool sym_eig(int n, const double* a, double* w, double* v);
void spark_side_seeds(int64_t seed, int64_t* user_seed, int64_t* item_seed);
void spark_initialize(const int32_t* ids_sorted, int64_t n, int rank, int64_t side_seed, int num_blocks,
                      float* out, int64_t ld);
void plan_shards(const int64_t* ptr, int64_t n, int world, int64_t* starts);
}  // namespace albedo
