/* the blocked LU order (8-column panels, swaps applied per panel, trailing
   rows updated with the panel's fmas in step order) gives bitwise the unblocked getf2 factors of
   k_solve.  gcc -O2 -ffp-contract=off tools/lu_block_check.c -lm && ./a.out */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define N 71
static int pivot(float A[N][N+1], int k){ float best=-1; int bi=N; for(int r=k;r<N;r++){float a=fabsf(A[r][k]); if(a>best){best=a;bi=r;}} return bi;}
static void unblocked(float A[N][N+1], int*piv){
  for(int k=0;k<N;k++){ int bi=pivot(A,k); piv[k]=bi; int p=bi<N?bi:k; float pv=bi<N?A[bi][k]:0.f;
    if(p!=k) for(int c=0;c<N;c++){float t=A[k][c];A[k][c]=A[p][c];A[p][c]=t;}
    float rc=1.0f/pv; for(int r=k+1;r<N;r++) A[r][k]=A[r][k]*rc;
    for(int r=k+1;r<N;r++) for(int c=k+1;c<N;c++) A[r][c]=fmaf(-A[r][k],A[k][c],A[r][c]); }
}
static void blocked(float A[N][N+1], int*piv){
  const int NB=8;
  for(int kb=0;kb<N;kb+=NB){ int ke=kb+NB<N?kb+NB:N;
    for(int k=kb;k<ke;k++){ int bi=pivot(A,k); piv[k]=bi; int p=bi<N?bi:k; float pv=bi<N?A[bi][k]:0.f;
      if(p!=k) for(int c=kb;c<ke;c++){float t=A[k][c];A[k][c]=A[p][c];A[p][c]=t;}
      float rc=1.0f/pv; for(int r=k+1;r<N;r++) A[r][k]=A[r][k]*rc;
      for(int r=k+1;r<N;r++) for(int c=k+1;c<ke;c++) A[r][c]=fmaf(-A[r][k],A[k][c],A[r][c]); }
    for(int c=0;c<N;c++){ if(c>=kb&&c<ke) continue;
      for(int k=kb;k<ke;k++){int p=piv[k]; if(p<N&&p!=k){float t=A[k][c];A[k][c]=A[p][c];A[p][c]=t;}}
      if(c>=ke) for(int k=kb;k<ke;k++) for(int r=k+1;r<ke;r++) A[r][c]=fmaf(-A[r][k],A[k][c],A[r][c]); }
    for(int r=ke;r<N;r++) for(int c=ke;c<N;c++){ float acc=A[r][c]; for(int k=kb;k<ke;k++) acc=fmaf(-A[r][k],A[k][c],acc); A[r][c]=acc; }
  }
}
int main(){ static float A[N][N+1],B[N][N+1]; int pa[N],pb[N]; int bad=0;
  srand(1);
  for(int t=0;t<200;t++){ for(int i=0;i<N;i++)for(int j=0;j<N;j++){A[i][j]=(float)rand()/RAND_MAX-0.5f; if(t%2==0&&i==j)A[i][j]+=3;} if(t%5==0) for(int j=0;j<N;j++) A[7][j]=A[3][j];
    memcpy(B,A,sizeof A); unblocked(A,pa); blocked(B,pb);
    if(memcmp(pa,pb,sizeof pa)) bad++; else for(int i=0;i<N;i++) if(memcmp(A[i],B[i],sizeof(float)*N)) {bad++;break;} }
  printf("mismatching matrices: %d of 200\n",bad); return bad!=0; }
