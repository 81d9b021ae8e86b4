// tests/cpp/from_json_check.cpp — drives ModelPredictiveControlAPI::from_json (solvempc_amd/cpp) on one
// JSON document for the CPU tests: `from_json_check '<json>' rows cols` prints "ok R C v00 v01 ..." or
// "<exception kind> <id> <what()>" (the reference's from_json, ModelPredictiveControlAPI.cpp:418-489,
// throws nlohmann::detail::type_error; json_lite mirrors that hierarchy).  Test program only.
#include <cstdio>
#include <cstdlib>
#include <iostream>

#include "../../solvempc_amd/cpp/mpc_api.hpp"

int main(int argc, char **argv)
{
    if (argc < 4) return 2;
    try {
        const json_lite::Value v = json_lite::parse(argv[1]);
        const mpcq::Matrix m = ModelPredictiveControlAPI::from_json(v, std::atoi(argv[2]), std::atoi(argv[3]));
        std::printf("ok %d %d", m.rows(), m.cols());
        for (int i = 0; i < m.rows(); i++)
            for (int j = 0; j < m.cols(); j++) std::printf(" %.17g", m(i, j));
        std::printf("\n");
    } catch (const json_lite::detail::type_error &e) {
        std::printf("type_error %d %s\n", e.id, e.what());
    } catch (const json_lite::detail::parse_error &e) {
        std::printf("parse_error %d %s\n", e.id, e.what());
    } catch (const json_lite::detail::out_of_range &e) {
        std::printf("out_of_range %d %s\n", e.id, e.what());
    }
    return 0;
}
