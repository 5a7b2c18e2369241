// Test driver for mdqtplasmasims_amd/csrc/mdqt_writer.hpp (tests/test_writer.py):
//   writer_check <in.bin> <out_dir>
// reads doubles from in.bin and writes them as "%lg\t...\n" rows of 6 through the FileWriter
// pool (four files, rows split round-robin by file) and through fprintf, for byte comparison.
#include "mdqt_writer.hpp"

#include <cstdio>
#include <memory>
#include <string>
#include <vector>

int main(int argc, char** argv) {
    if (argc != 3) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 3;
    auto x = std::make_shared<std::vector<double>>();
    double v;
    while (fread(&v, sizeof v, 1, f) == 1) x->push_back(v);
    fclose(f);
    const std::string d = argv[2];
    {
        mdqt::FileWriter w(4);
        for (int k = 0; k < 4; ++k)
            w.submit(d + "/async" + std::to_string(k) + ".dat", "w", [x, k](mdqt::LgText& t) {
                for (size_t i = (size_t)k * 6; i + 6 <= x->size(); i += 24) {
                    for (int c = 0; c < 6; ++c) { t.num((*x)[i + c]); t.ch('\t'); }
                    t.ch('\n');
                }
            });
        std::string err;
        if (w.flush(&err)) { fprintf(stderr, "%s\n", err.c_str()); return 4; }
        w.submit(d + "/no/such/dir/x.dat", "w", [](mdqt::LgText& t) { t.num(1.0); });
        if (w.flush(&err) == 0) return 5;                         // the error must surface
    }
    for (int k = 0; k < 4; ++k) {
        FILE* g = fopen((d + "/printf" + std::to_string(k) + ".dat").c_str(), "w");
        for (size_t i = (size_t)k * 6; i + 6 <= x->size(); i += 24) {
            const double* p = x->data() + i;
            fprintf(g, "%lg\t%lg\t%lg\t%lg\t%lg\t%lg\t\n", p[0], p[1], p[2], p[3], p[4], p[5]);
        }
        fclose(g);
    }
    return 0;
}
