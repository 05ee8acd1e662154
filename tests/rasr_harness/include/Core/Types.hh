// TEST DOUBLE (tests/rasr_harness/include/README): RASR's integer / float aliases and Core::Type
#pragma once
#include <cstdint>
#include <limits>
typedef int8_t   s8;
typedef uint8_t  u8;
typedef int16_t  s16;
typedef uint16_t u16;
typedef int32_t  s32;
typedef uint32_t u32;
typedef int64_t  s64;
typedef uint64_t u64;
typedef float    f32;
typedef double   f64;
namespace Core {
template <class T>
struct Type {
    static constexpr T max = std::numeric_limits<T>::max();
    static constexpr T min = std::numeric_limits<T>::lowest();
};
}  // namespace Core
