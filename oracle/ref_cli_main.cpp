/* ref_cli_main.cpp — TEST/MEASUREMENT INFRASTRUCTURE: entry point of the plain
 * reference x265 1.9 CLI (x265.cpp compiled with -Dmain=x265_cli_main, see
 * oracle/Makefile x265ref), no provider change: x265_setup_primitives fills the
 * C table itself (primitives.cpp:228-249).  Used as bench.py's CPU baseline.
 */
int x265_cli_main(int argc, char** argv);

int main(int argc, char** argv) { return x265_cli_main(argc, argv); }
