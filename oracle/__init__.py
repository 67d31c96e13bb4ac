# Test infrastructure only (see oracle/oracle.cpp header).
