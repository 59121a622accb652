// Thread churn without any GPU call: 8 threads each start and join `n`
// short-lived threads that allocate and free heap blocks, as
// tests/cpp/thread_exit_check.cpp's maskers do (diagnostic for a heap check
// that fired at thread shutdown on the GPU box).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

int main(int argc, char** argv)
{
    const int n = argc > 1 ? std::atoi(argv[1]) : 500;
    std::vector<std::thread> outer;
    for (int m = 0; m < 8; ++m)
        outer.emplace_back([n, m] {
            for (int g = 0; g < n; ++g) {
                std::thread t([m, g] {
                    std::vector<std::string> v;
                    for (int i = 0; i < 64; ++i) v.emplace_back((size_t)(1 + (m * 131 + g * 7 + i) % 9000), 'x');
                });
                t.join();
            }
        });
    for (auto& t : outer) t.join();
    std::printf("{\"threads\": %d, \"ok\": true}\n", 8 * n);
    return 0;
}
