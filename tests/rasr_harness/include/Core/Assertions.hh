// TEST DOUBLE: require / verify / ensure abort with a message (src/Core/Assertions.hh semantics)
#pragma once
#include <cstdio>
#include <cstdlib>
#define HARNESS_ASSERT(kind, c)                                                                   \
    do {                                                                                          \
        if (!(c)) {                                                                               \
            std::fprintf(stderr, "%s failed: %s (%s:%d)\n", kind, #c, __FILE__, __LINE__);          \
            std::abort();                                                                         \
        }                                                                                         \
    } while (0)
#define require(c) HARNESS_ASSERT("require", c)
#define require_(c) HARNESS_ASSERT("require", c)
#define verify(c) HARNESS_ASSERT("verify", c)
#define ensure(c) HARNESS_ASSERT("ensure", c)
#define require_eq(a, b) require((a) == (b))
#define require_lt(a, b) require((a) < (b))
