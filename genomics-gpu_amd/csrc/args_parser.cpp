// args_parser.cpp — Parameters (include/args_parser.h).  Same defaults, options,
// error behaviour and printout as Non-CDP/GASAL2/src/args_parser.cpp:8-250;
// "-y banded" is accepted as well (the reference cannot select BANDED from the
// command line).
#include "../../include/args_parser.h"

#include <string>

Parameters::Parameters(int argc_, char **argv_)
    : sa(1), sb(4), gapo(6), gape(1), start_pos(WITHOUT_START), print_out(0), n_threads(1), k_band(0),
      secondBest(FALSE), isPacked(false), isReverseComplement(false), semiglobal_skipping_head(TARGET),
      semiglobal_skipping_tail(TARGET), algo(UNKNOWN), argc(argc_), argv(argv_) {}

Parameters::~Parameters() {
    query_batch_fasta.close();
    target_batch_fasta.close();
}

void Parameters::print() {
    std::cerr << "sa=" << sa << " , sb=" << sb << " , gapo=" << gapo << " , gape=" << gape << std::endl;
    std::cerr << "start_pos=" << start_pos << " , print_out=" << print_out << " , n_threads=" << n_threads << std::endl;
    std::cerr << "semiglobal_skipping_head=" << semiglobal_skipping_head
              << " , semiglobal_skipping_tail=" << semiglobal_skipping_tail << " , algo=" << algo << std::endl;
    std::cerr << std::boolalpha << "isPacked = " << isPacked << " , secondBest = " << secondBest << std::endl;
    std::cerr << "query_batch_fasta_filename=" << query_batch_fasta_filename
              << " , target_batch_fasta_filename=" << target_batch_fasta_filename << std::endl;
}

void Parameters::failure(fail_type f) {
    if (f == NOT_ENOUGH_ARGS)
        std::cerr << "Not enough Parameters. Required: -y AL_TYPE file1.fasta file2.fasta. See help (--help, -h) for "
                     "usage. "
                  << std::endl;
    else if (f == WRONG_ARG)
        std::cerr << "Wrong argument. See help (--help, -h) for usage. " << std::endl;
    else if (f == WRONG_FILES)
        std::cerr << "File error: either a file doesn't exist, or cannot be opened." << std::endl;
    exit(1);
}

void Parameters::help() {
    std::cerr << "Usage: ./test_prog.out [-a] [-b] [-q] [-r] [-s] [-t] [-p] [-n] [-y] <query_batch.fasta> "
                 "<target_batch.fasta>"
              << std::endl;
    std::cerr << "Options: -a INT    match score [" << sa << "]" << std::endl;
    std::cerr << "         -b INT    mismatch penalty [" << sb << "]" << std::endl;
    std::cerr << "         -q INT    gap open penalty [" << gapo << "]" << std::endl;
    std::cerr << "         -r INT    gap extension penalty [" << gape << "]" << std::endl;
    std::cerr << "         -s        find the start position" << std::endl;
    std::cerr << "         -t        compute traceback. With this option enabled, \"-s\" has no effect as start "
                 "position will always be computed with traceback"
              << std::endl;
    std::cerr << "         -p        print the alignment results" << std::endl;
    std::cerr << "         -n INT    Number of threads [" << n_threads << "]" << std::endl;
    std::cerr << "         -y AL_TYPE       Alignment type . Must be \"local\", \"semi_global\", \"global\", \"ksw\" "
                 "(or \"banded\")"
              << std::endl;
    std::cerr << "         -x HEAD TAIL     specifies, for semi-global alignment, wha should be skipped for heads and "
                 "tails of the sequences. (NONE, QUERY, TARGET, BOTH)"
              << std::endl;
    std::cerr << "         -k INT    Band width in case \"banded\" is selected." << std::endl;
    std::cerr << "         --help, -h : displays this message." << std::endl;
    std::cerr << "         --second-best   displays second best score (WITHOUT_START only)." << std::endl;
    std::cerr << "Single-pack multi-Parameters (e.g. -sp) is not supported." << std::endl;
    std::cerr << "		  " << std::endl;
}

static bool parse_source(const std::string &s, data_source *out) {
    if (s == "NONE") *out = NONE;
    else if (s == "TARGET") *out = TARGET;
    else if (s == "QUERY") *out = QUERY;
    else if (s == "BOTH") *out = BOTH;
    else return false;
    return true;
}

void Parameters::parse() {
    for (int c = 1; c < argc; c++) {
        const std::string a(argv[c]);
        if (a == "--help" || a == "-h") { help(); exit(0); }
    }
    if (argc < 4) failure(NOT_ENOUGH_ARGS);
    int c = 1;
    for (; c < argc - 2; c++) {
        const std::string cur(argv[c]);
        if (cur.size() >= 2 && cur[0] == '-' && cur[1] == '-') {
            if (cur == "--help") { help(); exit(0); }
            if (cur == "--second-best") secondBest = TRUE;
            continue;
        }
        if (cur.empty() || cur[0] != '-') failure(WRONG_ARG);
        if (cur.size() > 2) failure(WRONG_ARG);
        auto next = [&]() -> std::string { return std::string(argv[++c]); };
        switch (cur.at(1)) {
            case 'y': {
                const std::string v = next();
                if (v == "local") algo = LOCAL;
                else if (v == "semi_global") algo = SEMI_GLOBAL;
                else if (v == "global") algo = GLOBAL;
                else if (v == "ksw") algo = KSW;
                else if (v == "banded") algo = BANDED;
                break;
            }
            case 'a': sa = std::stoi(next()); break;
            case 'b': sb = std::stoi(next()); break;
            case 'q': gapo = std::stoi(next()); break;
            case 'r': gape = std::stoi(next()); break;
            case 's': start_pos = WITH_START; break;
            case 't': start_pos = WITH_TB; break;
            case 'p': print_out = 1; break;
            case 'n': n_threads = std::stoi(next()); break;
            case 'k': k_band = std::stoi(next()); break;
            case 'x':
                if (!parse_source(next(), &semiglobal_skipping_head)) failure(WRONG_ARG);
                if (!parse_source(next(), &semiglobal_skipping_tail)) failure(WRONG_ARG);
                break;
            default: break;
        }
    }
    query_batch_fasta_filename = std::string(argv[c]);
    target_batch_fasta_filename = std::string(argv[c + 1]);
    fileopen();
}

void Parameters::fileopen() {
    query_batch_fasta.open(query_batch_fasta_filename, std::ifstream::in);
    if (!query_batch_fasta) failure(WRONG_FILES);
    target_batch_fasta.open(target_batch_fasta_filename);
    if (!target_batch_fasta) failure(WRONG_FILES);
}
