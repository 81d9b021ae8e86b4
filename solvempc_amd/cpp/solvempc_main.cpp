// solvempc_amd/cpp/solvempc_main.cpp — the reference's solver.cpp control loop (src/solver.cpp:13-80)
// with the serial port (out of scope: hardware I/O) replaced by a replay stream in the same wire
// format: every input line is one "serial message"; lines longer than 30 bytes are parsed as
// "dt x0 x1 x2 x3" into float (SerialPort.cpp:106-139, incl. its float[5] buffer), shorter ones are
// bad reads that resend the last U (solver.cpp:69-73).  Each output line is what writePort sends:
// the first sizeof(char*) = 8 characters of std::to_string(U) (SerialPort.cpp:162-166), one per line,
// to stdout or to the -o file (the "serial port" side, kept apart from the -v log).
//
//   solvempc [-v] [-c ./config/MPC_API.json] [-N 15] [-i messages.txt] [-o wire.txt]
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>

#include "mpc_api.hpp"

static bool parse_message(const std::string &line, double &dt, mpcq::Matrix &X)
{
    if (line.size() + 1 <= 30) return false;  // readPort: num_bytes > 30 (the newline counts)
    float ref[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    char buf[256];
    std::strncpy(buf, line.c_str(), sizeof(buf) - 1);
    buf[sizeof(buf) - 1] = '\0';
    char *ptr = std::strtok(buf, " ");
    for (int index = 0; index < 5; index++) {
        const double t = ptr ? std::atof(ptr) : 0.0;
        if (t != 0) ref[index] = (float)t;
        ptr = std::strtok(nullptr, " ");
    }
    dt = ref[0];
    for (int i = 0; i < 4; i++) X(i) = ref[i + 1];
    return true;
}

static std::string wire(double u)
{
    return std::to_string(u).substr(0, sizeof(char *));
}

int main(int argc, char **argv)
{
    std::cout << "\n\n[solveMPC]\tStarting MPC solver.\n\n" << std::endl;
    bool verbose = false;
    if (cmdOptionExists(argv, argv + argc, "-v")) {
        verbose = true;
        std::cout << "[solveMPC]\tVerbose output on." << std::endl;
    }
    const char *cfg = getCmdOption(argv, argv + argc, "-c");
    const char *hz = getCmdOption(argv, argv + argc, "-N");
    const char *in = getCmdOption(argv, argv + argc, "-i");
    const char *outp = getCmdOption(argv, argv + argc, "-o");
    ModelPredictiveControlAPI mpc(verbose, cfg ? cfg : "./config/MPC_API.json", hz ? std::atoi(hz) : mpcWindow);
    if (!mpc.solverFlag) return 1;

    std::ifstream file;
    if (in) file.open(in);
    if (in && !file) {
        std::cerr << "[solveMPC]\tcannot open " << in << std::endl;
        return 1;
    }
    std::istream &src = in ? static_cast<std::istream &>(file) : std::cin;
    std::ofstream wfile;
    if (outp) wfile.open(outp);
    std::ostream &wire_out = outp ? static_cast<std::ostream &>(wfile) : std::cout;
    std::cout << "----------------------------------------------------\n"
                 "-------------- Entering control loop. --------------\n"
                 "----------------------------------------------------" << std::endl;
    std::string line;
    double dt_msg = 0.0;  // readPort takes dt by value: mpc.dt never changes (SerialPort.cpp:142)
    while (std::getline(src, line)) {
        if (parse_message(line, dt_msg, mpc.X)) {
            if (mpc.verbose)  // (SerialPort.cpp:150; the message keeps its newline)
                std::cout << "\n[SerialPort]\tRead " << line.size() + 1 << " bytes. Received message: " << line << "\n";
            if (!mpc.controllerStep()) return 1;
            if (mpc.verbose) {  // (solver.cpp:53-57)
                std::cout << "[solveMPC]\tCurrent state: " << mpc.X.transpose() << std::endl;
                std::cout << "[solveMPC]\tControl output: " << mpc.U.transpose() << std::endl;
            }
        }
        wire_out << wire(mpc.U(0)) << std::endl;  // writePort(mpc.U); a bad read resends the last U (:69-73)
    }
    return 0;
}
