// tests/emu/occ_check.cpp — TEST ONLY: the library's .bwt loader + HBM occ re-layout
// (desamba-so_amd/csrc/index_load.c dsb_index_load_bwt) and the device occ (dsb_occ,
// desamba-so_amd/csrc/gpu/dsb_core.h, compiled for the host) on the rows of a file, in the layout
// of oracle/_ref/bigbwt occ (the reference's own occ on the same index):
//     occ_check DIR DOLLOR_POS ROWS OUT      7 u64 per row: occ(r, c) c = 0..4, occ(r, 0xff), its symbol
// Exit status 2 with the loader's message when the re-layout rejects the file.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
extern "C" {
#include "../../desamba-so_amd/csrc/dsb_host.h"
}
#include "../../desamba-so_amd/csrc/gpu/dsb_core.h"

extern "C" int dsb_host_threads(void) { return 4; } /* pool.c is not linked here */

int main(int argc, char **argv)
{
	if (argc != 5) {
		fprintf(stderr, "usage: occ_check DIR DOLLOR_POS ROWS OUT\n");
		return 1;
	}
	static dsb_index ix;
	char err[512] = "";
	if (dsb_index_load_bwt(&ix, argv[1], 0, err, sizeof(err))) {
		fprintf(stderr, "%s\n", err);
		return 2;
	}
	dsb_dindex_t d;
	memset(&d, 0, sizeof(d));
	d.occ = ix.occ;
	d.occ_super = ix.occ_super;
	d.n_occ_line = ix.n_occ_line;
	memcpy(d.dollar_row, ix.dollar_row, sizeof(d.dollar_row));
	d.n_dollar = ix.n_dollar;
	memcpy(d.rank, ix.rank, sizeof(d.rank));
	d.dollor_pos = strtoull(argv[2], 0, 10);
	FILE *f = fopen(argv[3], "rb");
	std::vector<uint64_t> rows;
	uint64_t r;
	while (fread(&r, 8, 1, f) == 1)
		rows.push_back(r);
	fclose(f);
	std::vector<uint64_t> out(7 * rows.size());
	for (size_t i = 0; i < rows.size(); i++) {
		for (int c = 0; c < 5; c++) {
			uint8_t cc = (uint8_t)c;
			out[7 * i + c] = dsb_occ(&d, rows[i], &cc);
		}
		uint8_t cf = 0xff;
		out[7 * i + 5] = dsb_occ(&d, rows[i], &cf);
		out[7 * i + 6] = cf;
	}
	f = fopen(argv[4], "wb");
	fwrite(out.data(), 8, out.size(), f);
	fclose(f);
	return 0;
}
